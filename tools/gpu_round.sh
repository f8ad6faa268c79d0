#!/bin/bash
# One GPU session of the round's final measurements (run under gpurun):
#   tools/gpu_round.sh TAG bench     bench.py lines: default (cfg2 + its extra legs) and cfg3/4/5
#   tools/gpu_round.sh TAG tests     pytest -m gpu + smoke()
#   tools/gpu_round.sh TAG stats     rocprofv3 --kernel-trace --stats of the default bench command
#   tools/gpu_round.sh TAG profile   per-leg kernel trace + FETCH_SIZE + WRITE_SIZE passes (tools/profile_r02.sh)
#   tools/gpu_round.sh TAG host      host-memory end to end (tools/e2e_host.py) and per-call latency (tools/bytes_latency.py)
#   tools/gpu_round.sh TAG pmc       SQ counters (tools/pmc_sq.sh: cfg2-cfg5, first_seen) and wide codes (tools/pmc_wide.sh)
# Every step has its own time limit and the steps are chained with &&.
set -e
TAG=$1
shift
ROUND=${ROUND:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $ROOT
for what in "$@"; do
  case $what in
    bench)
      timeout -k 10 420 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
      for W in cfg3 cfg4 cfg5; do
        timeout -k 10 300 python -u bench.py --workload $W --no-cpu > $OUT/bench_$W.json 2> $OUT/bench_$W.err
      done ;;
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 ;;
    host)
      timeout -k 10 420 python -u tools/e2e_host.py > $OUT/e2e_host.log 2>&1
      timeout -k 10 420 python -u tools/bytes_latency.py > $OUT/bytes_latency.log 2>&1 ;;
    stats)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
        -d $OUT/stats -o st -- python3 $ROOT/bench.py --no-cpu > $OUT/stats_bench.json 2> $OUT/stats_bench.err)
      # keep the --stats summary, drop the per-dispatch trace (gpurun copies back <= 64 MiB)
      find $OUT/stats -name "*kernel_trace.csv" -delete ;;
    profile)
      tools/profile_r02.sh $TAG/prof
      # summarised here (the raw traces and counter dumps exceed gpurun's 64 MiB copy-back)
      python3 tools/legs_summary.py $TAG/prof $ROUND > $OUT/legs_summary.log 2>&1 || true
      python3 tools/bench_vs_trace.py $TAG/prof $ROUND > $OUT/${ROUND}_bench_vs_trace.txt 2>&1 || true
      mkdir -p $OUT/summary
      cp profiles/${ROUND}_legs_*.json profiles/${ROUND}_cfg*_kernel_stats.csv $OUT/summary/ || true
      rm -rf $OUT/prof ;;
    pmc)
      for W in cfg2 cfg3 cfg4 cfg5 first_seen; do tools/pmc_sq.sh $W $TAG/sq; done
      tools/pmc_wide.sh $TAG/wide
      python3 tools/pmc_sq_summary.py $TAG/sq $ROUND cfg2 cfg3 cfg4 cfg5 first_seen > $OUT/pmc_sq_summary.log 2>&1 || true
      python3 tools/pmc_wide_summary.py $TAG/wide $ROUND > $OUT/pmc_wide_summary.log 2>&1 || true
      mkdir -p $OUT/summary
      cp profiles/pmc_sq_summary.json profiles/${ROUND}_pmc_sq.json profiles/${ROUND}_wide_rooflines.json $OUT/summary/ || true
      find $OUT/wide/kt -name "*kernel_stats.csv" -exec cp {} $OUT/summary/${ROUND}_wide_kernel_stats.csv \;
      rm -rf $OUT/sq $OUT/wide ;;
  esac
  echo "gpu_round $what done"
done
