# round 5, session q7: phase length of the 2-wave plane-sharing form by tile
# height: var1 (2 inputs for 9-10-row tiles, 4 below) against base (2 always);
# cfg4's fresh-pattern decodes (11-16 rows: 6-8-row tiles) and first-seen leg.
set -o pipefail
O=gpurun_out/r05q7
mkdir -p $O
(cd scratch/var1 && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py) \
  > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in base var1; do
    d=scratch/$t
    (cd $d && timeout -k 10 300 python -u bench.py --workload cfg4 --no-cpu --no-extra --steps 10) > $O/cfg4_${t}_$i.json 2> $O/cfg4_${t}_$i.err \
      || { echo cfg4-$t-failed; tail -20 $O/cfg4_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/33,12/30,16/30,20/36,10/26 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05q7/cfg4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    x, fs = d["decode_fresh_pattern"], d.get("first_seen_decode", {})
    print(f.split("/")[-1], d["value"], "fresh", x["ms_mean"], x["hbm_GBps_mean"], "first_seen", fs.get("first_seen", {}).get("ms_mean"))
PY
