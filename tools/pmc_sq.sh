#!/bin/bash
# Issue-side counters of one bench workload's kernels (instruction cache, wave states),
# each pass in its own rocprofv3 run: tools/pmc_sq.sh WORKLOAD TAG
set -e
W=${1:-cfg4}
TAG=${2:-sq}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out/$TAG/$W
mkdir -p $OUT
ARGS="--workload $W --steps 3 --warmup 1 --no-cpu --no-extra"
timeout -s KILL 240 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/ic -o ic -- python3 $ROOT/bench.py $ARGS > $OUT/ic.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $OUT/sq -o sq -- python3 $ROOT/bench.py $ARGS > $OUT/sq.log 2>&1
echo pmc-sq-done
