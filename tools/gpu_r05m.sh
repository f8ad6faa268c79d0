# round 5, session m: tile policy for 17-20-row matapply_bsr launches on the
# first_seen leg (cfg4's 20-row decodes): shipped (2 waves x 10 rows) against
# var1 (4 waves x 5 rows) and var2 (4 waves x 5 rows, combinations shared)
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
for i in 1 2; do
  for t in new var1 var2; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/40,20/60,12/30,30/70 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
