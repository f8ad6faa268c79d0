# round 5, session o2: wave priority of matapply_bsr's LDS-phase load stage
# (s_setprio 3 while a wave loads and transposes a phase's inputs, 0 for the
# routine calls) against the previous tree (scratch/base) and var1 (priority 1);
# parity first
set -o pipefail
O=gpurun_out/r05o2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -2 $O/pytest_bsr.log
for i in 1 2; do
  for t in new base var1; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/40,20/60,12/30,30/70 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
