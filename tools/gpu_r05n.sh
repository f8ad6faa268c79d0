# round 5, session n: wide codes with many rows on the LDS-phase form with shared
# combinations (var1: every k > 32, r > 10 launch on lds,tbl; var2: the same
# with 8-row tiles always) against the shipped ks row groups
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
for i in 1 2; do
  for t in new var1 var2; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 200/256,64/112,160/256,100/200,128/256 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
