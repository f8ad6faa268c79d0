# round 5, session r: north-star batch (256 x 1 MiB K=3/M=10 object-major) with
# FEC_FLAG_ROW_PADDING (rows run to their next 128-byte line, as the main bench's
# calls do), stores nt (shipped) and nt sc1 (scratch/sc1), against no padding
set -o pipefail
O=gpurun_out/r05r
mkdir -p $O
for i in 1 2; do
  for t in new sc1; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    for p in pad nopad; do
      a=""; [ $p = pad ] && a="--row-padding"
      (cd $d && timeout -k 10 300 python -u $GRAFT_REPO_ROOT/tools/batch_ab.py --stripes 256 --rounds 1 $a) > $O/batch_${t}_${p}_$i.json 2> $O/batch_${t}_${p}_$i.err \
        || { echo batch-$t-$p-failed; tail -20 $O/batch_${t}_${p}_$i.err; exit 1; }
    done
  done
done
python tools/r05_summary.py $O
