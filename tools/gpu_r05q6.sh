# round 5, session q6: matapply_bsr's one-wave (solo) form stages its inputs in
# 8 KiB of LDS per wave by LDS-DMA, a phase of 2 inputs loading while the wave
# walks the previous one (bsr_walk_lds), instead of loading two inputs ahead
# into registers; against the shipped tree (scratch/base); parity first
set -o pipefail
O=gpurun_out/r05q6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu --no-extra --no-first-seen --steps 10) > $O/cfg3_${t}_$i.json 2> $O/cfg3_${t}_$i.err \
      || { echo cfg3-$t-failed; tail -20 $O/cfg3_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 10/16,20/30,16/24,32/40,12/16,10/13 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05q6/cfg3_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    x = d["decode_fresh_pattern"]
    print(f.split("/")[-1], d["value"], "fresh", x["ms_mean"], x["hbm_GBps_mean"], x["kernels"])
PY
