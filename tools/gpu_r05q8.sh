# round 5, session q8: phase lengths once more -- var1: matapply_bsr's 2-wave
# plane-sharing form in phases of 3 (shipped: 2); var2: the JIT's double-buffered
# phases of 6 (shipped: 4); base: the shipped tree.  cfg4 (first-seen and
# fresh-pattern decodes on matapply_bsr, the compiled r = 20 decode) and the
# 2-wave wide shapes.  Parity of both variants first.
set -o pipefail
O=gpurun_out/r05q8
mkdir -p $O
(cd scratch/var1 && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py) \
  > $O/pytest_var1.log 2>&1 || { echo pytest-var1-failed; tail -30 $O/pytest_var1.log; exit 1; }
(cd scratch/var2 && timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_jit.py) \
  > $O/pytest_var2.log 2>&1 || { echo pytest-var2-failed; tail -30 $O/pytest_var2.log; exit 1; }
tail -1 $O/pytest_var1.log; tail -1 $O/pytest_var2.log
for i in 1 2; do
  for t in base var1 var2; do
    d=scratch/$t
    (cd $d && timeout -k 10 300 python -u bench.py --workload cfg4 --no-cpu --no-extra --steps 10) > $O/cfg4_${t}_$i.json 2> $O/cfg4_${t}_$i.err \
      || { echo cfg4-$t-failed; tail -20 $O/cfg4_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/33,12/30,16/30,20/36 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05q8/cfg4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    x, fs = d["decode_fresh_pattern"], d["first_seen_decode"]
    print(f.split("/")[-1], d["value"], "dec", d["decode_roofline"]["launch_ms"], "fresh", x["ms_mean"], "first_seen", fs["first_seen"]["ms_mean"], "jit", fs["jit"]["ms_mean"])
PY
