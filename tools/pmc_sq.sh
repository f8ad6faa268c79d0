#!/bin/bash
# Issue-side and LDS counters of one bench workload's kernels, each pass in its
# own rocprofv3 run: tools/pmc_sq.sh WORKLOAD TAG [extra bench args]
# (tools/pmc_sq_summary.py TAG ROUND WORKLOAD... turns them into profiles/pmc_sq_summary.json)
set -e
W=${1:-cfg4}
TAG=${2:-sq}
shift 2 || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out/$TAG/$W
mkdir -p $OUT
ARGS="--workload $W --steps 3 --warmup 1 --no-cpu --no-extra $*"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/sq -o sq -- python3 $ROOT/bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o lds -- python3 $ROOT/bench.py $ARGS > $OUT/lds.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sca -o sca -- python3 $ROOT/bench.py $ARGS > $OUT/sca.log 2>&1
echo pmc-sq-done $W
