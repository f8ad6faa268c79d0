# round 5, session q2: double-buffered LDS-DMA phases in the JIT generator
# (bitslice.cpp: a phase's inputs straight into LDS, transposed in place, the
# next phase loading while the waves walk the current one) and in matapply_bsr's
# plane-sharing form (phases of 4).  Trees: new (JIT phases of 4 where the
# inputs do not all fit, else one DMA phase; bsr phases of 4), base (previous
# tree: register-loaded phases of 8 in both), var1 (JIT phases of 4 always:
# K=20/M=60's r = 40 encode too), var2 (bsr phases of 2).  Parity first.
set -o pipefail
O=gpurun_out/r05q2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_jit.py \
  > $O/pytest.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for t in new base var1 var2; do
    if [ $t = new ]; then d=.; else d=scratch/$t; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 300 python -u bench.py --workload cfg4 --no-cpu --no-extra --no-first-seen) > $O/cfg4_${t}_$i.json 2> $O/cfg4_${t}_$i.err \
      || { echo cfg4-$t-failed; tail -20 $O/cfg4_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 400 python -u tools/wide_bench.py --shapes 20/40,20/60,30/70,12/30,20/33 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python tools/r05_summary.py $O
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05q2/cfg4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r, dr = d["roofline"], d.get("decode_roofline", {})
    print(f.split("/")[-1], d["value"], r["kernel"][:40], r["launch_ms"], r["frac"], dr.get("kernel", "")[:40], dr.get("launch_ms"), dr.get("frac"))
PY
