# round 5, session q9: tiles of cfg4's 20-row first-seen decodes on the
# DMA-staged phases: var1 (4 waves x 5 rows, as small launches already run)
# against the shipped 2 waves x 10 rows (base); parity of var1 first
set -o pipefail
O=gpurun_out/r05q9
mkdir -p $O
(cd scratch/var1 && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py -k "not argument_and_table") \
  > $O/pytest_var1.log 2>&1 || { echo pytest-var1-failed; tail -30 $O/pytest_var1.log; exit 1; }
tail -1 $O/pytest_var1.log
for i in 1 2 3; do
  for t in base var1; do
    d=scratch/$t
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
