# round 5, session p5: phase length of the double-buffered LDS-DMA form for
# 4-wave workgroups: 8 inputs (shipped candidate) against var1 (4 inputs)
set -o pipefail
O=gpurun_out/r05p5
mkdir -p $O
for i in 1 2; do
  for t in new var1; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/40,20/60,30/70,24/48,16/40 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
