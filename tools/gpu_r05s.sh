# round 5, session s: what the row end costs on the north-star batch shape
# (256 stripes per launch, rows 256-byte aligned): block size not a multiple of
# 16 (349,526: the last 16-byte chunk overlaps its neighbour), a multiple of 16
# but not of 128 (349,520: the row ends mid-line), a multiple of 128 (349,568),
# and 349,526 with FEC_FLAG_ROW_PADDING
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
for i in 1 2; do
  for v in 349526 349520 349568 pad; do
    a="--sz $v"; [ $v = pad ] && a="--row-padding"
    timeout -k 10 300 python -u tools/batch_ab.py --stripes 256 --rounds 1 $a > $O/batch_${v}_$i.json 2> $O/batch_${v}_$i.err \
      || { echo batch-$v-failed; tail -20 $O/batch_${v}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
