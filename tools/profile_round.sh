#!/bin/bash
# Profile the default bench workload on the GPU box with rocprofv3:
#   1. kernel trace + stats (per-kernel average durations),
#   2. FETCH_SIZE and 3. WRITE_SIZE PMC counters, each in its own pass
#      (MI355X_MICROARCH.md "rocprofv3 PMC slots": they do not fit one pass).
# Output under gpurun_out/$TAG/; tools/pmc_summary.py turns it into profiles/.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 20 --warmup 3 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o kt -- python3 $ROOT/bench.py $ARGS > $OUT/ktrace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o f -- python3 $ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o w -- python3 $ROOT/bench.py $ARGS > $OUT/write.log 2>&1
echo profile-done
