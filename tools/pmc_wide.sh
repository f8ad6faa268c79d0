#!/bin/bash
# Counters of the wide-code kernels (tools/wide_bench.py, shipped variant), each pass its
# own rocprofv3 run: tools/pmc_wide.sh TAG  ->  gpurun_out/TAG/{kt,sq,lds}
# (tools/pmc_wide_summary.py TAG ROUND writes profiles/<ROUND>_wide_rooflines.json)
set -e
TAG=${1:-wide}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
ARGS="--variants shipped --launches 10 ${SHAPES:+--shapes $SHAPES}"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $ROOT/tools/wide_bench.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- python3 $ROOT/tools/wide_bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/lds -o lds -- python3 $ROOT/tools/wide_bench.py $ARGS > $OUT/lds.log 2>&1
echo pmc-wide-done
