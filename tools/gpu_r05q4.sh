# round 5, session q4: matapply_bsr's combination-sharing form (8-wave
# workgroups, wide codes) stages each phase's inputs with LDS-DMA while the
# waves walk the previous phase, against the previous tree (scratch/base:
# register loads at the start of each phase); parity first
set -o pipefail
O=gpurun_out/r05q4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 128/256,160/256,64/112,30/70,40/88 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
