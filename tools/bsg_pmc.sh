#!/bin/bash
# Counter passes over tools/bsg_probe.py (one rocprofv3 run per pass):
#   tools/bsg_pmc.sh TAG KIND [OP]     e.g. tools/bsg_pmc.sh bsgpmc bsg dec
set -e
TAG=${1:-bsgpmc}
KIND=${2:-bsg}
OP=${3:-dec}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out/$TAG/$KIND-$OP
mkdir -p $OUT
ARGS="--kind $KIND --op $OP --reps 5"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $ROOT/tools/bsg_probe.py $ARGS > $OUT/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/a -o a -- python3 $ROOT/tools/bsg_probe.py $ARGS > $OUT/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_LDS_ADDR_CONFLICT --output-format csv -d $OUT/b -o b -- python3 $ROOT/tools/bsg_probe.py $ARGS > $OUT/b.log 2>&1
echo bsg-pmc-done $KIND $OP
