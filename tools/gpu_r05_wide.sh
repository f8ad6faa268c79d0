# round 5 final tree: counters of the shipped wide-code kernels (tools/pmc_wide.sh),
# summarised on the box into gpurun_out/$TAG/out/
set -o pipefail
T=${TAG:-r05ww}
SHAPES=94/100,64/112,128/256,160/256,200/256,255/256 bash tools/pmc_wide.sh $T || { echo pmc-wide-failed; exit 1; }
mkdir -p gpurun_out/$T/out
python tools/pmc_wide_summary.py $T r05 > gpurun_out/$T/out/summary.log 2>&1
cp profiles/r05_wide_rooflines.json profiles/r05_wide_kernel_stats.csv gpurun_out/$T/out/ 2>/dev/null
cp gpurun_out/$T/kt.log gpurun_out/$T/out/wide_bench_kt.log 2>/dev/null
rm -rf gpurun_out/$T/kt gpurun_out/$T/sq gpurun_out/$T/lds
echo wide-done
