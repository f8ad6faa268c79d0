# round 5, session t: the default bench line with the row-padding contract on the
# batched and first-seen legs, twice; then cfg4 (decode_fresh leg)
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/bench_cfg2_$i.json 2> $O/bench_cfg2_$i.err || { echo bench-failed; tail $O/bench_cfg2_$i.err; exit 1; }
  python tools/show_bench.py $O/bench_cfg2_$i.json
done
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo bench4-failed; tail $O/bench_cfg4.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r05t/bench_cfg2_1.json", "gpurun_out/r05t/bench_cfg2_2.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print({k: (v["frac_of_peak"], v["ms_per_launch"]) for k, v in d["batched_1MiB"]["layouts"].items()})
d = json.loads(open("gpurun_out/r05t/bench_cfg4.json").read().strip().splitlines()[-1])
print("cfg4", d["value"], d.get("decode_fresh"))
PY
