# round 5, session o: wide-code policy (8-row tiles always; ks only where the
# LDS-phase workgroups would not give every CU one) against the previous tree
set -o pipefail
O=gpurun_out/${TAG:-r05o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_bsg.py \
  > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -2 $O/pytest_bsr.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/base; fi
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 200/256,64/112,160/256,100/200,128/256,96/128,80/160,40/60,48/64 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
