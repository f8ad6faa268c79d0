#!/bin/bash
# Round-2 profile of bench.py workloads on the GPU box (rocprofv3), leg by leg:
#   1. kernel trace (+ --stats), 2. FETCH_SIZE pass, 3. WRITE_SIZE pass, each in
#   its own run with the same arguments, each run writing its own launch
#   sequence (bench.py --legs-out) so tools/trace_legs.py can pair the
#   dispatches of every pass with bench.py's legs (timed loop, warm / cold
#   back-to-back launches, fresh-pattern decodes).
# usage: tools/profile_r02.sh TAG [WORKLOAD ...]   (default: cfg2 cfg3 cfg4 cfg5)
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
  EXTRA=""
  [ "$W" = "cfg2" ] || EXTRA="--no-extra"
  ARGS="--workload $W --steps 20 --warmup 3 --no-cpu $EXTRA"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o kt -- python3 $ROOT/bench.py $ARGS --legs-out $OUT/legs_kt.json > $OUT/ktrace.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o f -- python3 $ROOT/bench.py $ARGS --legs-out $OUT/legs_f.json > $OUT/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o w -- python3 $ROOT/bench.py $ARGS --legs-out $OUT/legs_w.json > $OUT/write.log 2>&1
  echo "profiled $W"
done
echo profile-done
