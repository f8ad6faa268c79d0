# round 5, session o3: s_setprio in the table form's load stage only
# (kBsrTblLoadPrio) against the previous tree (scratch/base) on the wide codes
# whose launches take the table form (128/256, 160/256: 8-wave combination-sharing
# workgroups; 30/70, 20/60 encode: 4 waves); parity first
set -o pipefail
O=gpurun_out/r05o3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -2 $O/pytest_bsr.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 128/256,160/256,30/70,20/60,64/112 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
