# round 5, session b: matapply_bsr register block at v8 and a 2-input load batch
# for 9-10 row tiles (bsr<10,lds> 144 -> 125 VGPRs, 4 waves per SIMD): parity, then
# A/B against the previous tree (scratch/base) on the first_seen leg and the
# generic (first-launch) wide shapes whose tiles are 9-10 rows
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -2 $O/pytest_bsr.log
for i in 1 2; do
  for t in new base; do
    if [ $t = new ]; then d=.; else d=scratch/base; fi
    (cd $d && timeout -k 10 300 python -u bench.py --workload first_seen) > $O/fs_${t}_$i.json 2> $O/fs_${t}_$i.err \
      || { echo fs-$t-failed; tail -20 $O/fs_${t}_$i.err; exit 1; }
    (cd $d && timeout -k 10 300 python -u tools/wide_bench.py --shapes 20/60,30/70,12/30 --variants generic --launches 10) \
      > $O/wide_${t}_$i.json 2> $O/wide_${t}_$i.err || { echo wide-$t-failed; tail -20 $O/wide_${t}_$i.err; exit 1; }
  done
done
python - <<'EOF'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05b/fs_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])["first_seen_decode"]
    print(f, d["first_seen"]["kernel"], d["first_seen"]["ms_mean"], d["first_seen"]["frac_of_peak"], "jit", d["jit"]["ms_mean"])
for f in sorted(glob.glob("gpurun_out/r05b/wide_*.json")):
    d = json.load(open(f))["shapes"]
    print(f, {s: (v["generic"]["encode"]["kernel"], v["generic"]["encode"]["ms"], v["generic"]["decode"]["kernel"],
                  v["generic"]["decode"]["ms"]) for s, v in d.items()})
EOF
