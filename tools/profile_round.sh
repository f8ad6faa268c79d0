#!/bin/bash
# Profile bench.py workloads on the GPU box with rocprofv3:
#   1. kernel trace + stats (per-kernel average durations),
#   2. FETCH_SIZE and 3. WRITE_SIZE PMC counters, each in its own pass
#      (MI355X_MICROARCH.md "rocprofv3 PMC slots": they do not fit one pass).
# usage: tools/profile_round.sh TAG [WORKLOAD ...]   (default: cfg2 cfg3 cfg4 cfg5)
# Output under gpurun_out/$TAG/<workload>/; tools/pmc_summary.py turns it into profiles/.
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
shift || true
WLS=${@:-cfg2 cfg3 cfg4 cfg5}
export TMPDIR=/tmp
cd /tmp
for W in $WLS; do
  OUT=$ROOT/gpurun_out/$TAG/$W
  mkdir -p $OUT
  # the same arguments in all three passes: tools/pmc_summary.py matches dispatches by order
  ARGS="--workload $W --steps 20 --warmup 3 --no-cpu --no-extra"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o kt -- python3 $ROOT/bench.py $ARGS > $OUT/ktrace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o f -- python3 $ROOT/bench.py $ARGS > $OUT/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o w -- python3 $ROOT/bench.py $ARGS > $OUT/write.log 2>&1
  echo "profiled $W"
done
echo profile-done
