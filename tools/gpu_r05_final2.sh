# round 5 final tree, part 2: per-leg kernel traces and PMC traffic of every
# BASELINE workload (tools/profile_r02.sh), then the issue-side counters
# (tools/pmc_sq.sh) of the same workloads and the first_seen leg.  The summaries
# are made on the box (the raw rocprofv3 output is too large to copy back) and
# left under gpurun_out/$TAG/out/ for profiles/.
set -o pipefail
P=${TAG:-r05p}
R=${ROUND:-r05}
bash tools/profile_r02.sh $P cfg2 cfg3 cfg4 cfg5 || { echo profile-failed; exit 1; }
for w in cfg2 cfg3 cfg4 cfg5 first_seen; do
  bash tools/pmc_sq.sh $w ${P}sq || { echo pmc-$w-failed; exit 1; }
done
mkdir -p gpurun_out/$P/out
python tools/legs_summary.py $P $R cfg2 cfg3 cfg4 cfg5 > gpurun_out/$P/out/legs_summary.log 2>&1
python tools/bench_vs_trace.py $P $R cfg2 cfg3 cfg4 cfg5 > gpurun_out/$P/out/${R}_bench_vs_trace.txt 2>&1
python tools/pmc_sq_summary.py ${P}sq $R cfg2 cfg3 cfg4 cfg5 first_seen > gpurun_out/$P/out/pmc_sq_summary.log 2>&1
cp profiles/${R}_legs_cfg*.json profiles/${R}_cfg*_kernel_stats.csv profiles/pmc_sq_summary.json profiles/${R}_pmc_sq.json gpurun_out/$P/out/ 2>/dev/null
for w in cfg2 cfg3 cfg4 cfg5; do cp gpurun_out/$P/$w/ktrace.log gpurun_out/$P/out/ktrace_$w.log; done
rm -rf gpurun_out/${P}sq gpurun_out/$P/cfg2 gpurun_out/$P/cfg3 gpurun_out/$P/cfg4 gpurun_out/$P/cfg5
du -sh gpurun_out
echo final2-done
