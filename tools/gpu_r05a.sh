# round 5, session a: matapply_bsr parity where it ships (full cfg3/cfg4 size,
# past the grid cap), then the default bench line with the first_seen_decode leg
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bsr.py \
  "tests/test_gpu_parity.py::test_config3_256mib_roundtrip" "tests/test_gpu_parity.py::test_config4_1024_stripes_of_1mib" \
  > $O/pytest_bsr.log 2>&1 || { echo pytest-failed; tail -30 $O/pytest_bsr.log; exit 1; }
tail -3 $O/pytest_bsr.log
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench-failed; tail -20 $O/bench_default.err; exit 1; }
python tools/show_bench.py $O/bench_default.json 2>/dev/null || tail -c 3000 $O/bench_default.json
