# round 5, session q5: combination sharing (8-wave workgroups only so far) for
# the 2- and 4-wave LDS-phase launches now that its phases are staged by
# LDS-DMA: var1 (nw >= 2: cfg4's first-seen decodes too), var2 (nw >= 4),
# against the shipped tree (base); timing only (the kept variant's parity runs after)
set -o pipefail
O=gpurun_out/r05q5
mkdir -p $O
for i in 1 2; do
  for t in base var1 var2; do
    d=scratch/$t
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/40,20/60,30/70,12/30,20/33 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
