# round 5: bsr / JIT GPU tests after the graph-capture guard and the JIT phase policy
set -o pipefail
O=gpurun_out/r05w2
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bsr.py tests/test_gpu_jit.py tests/test_gpu_bsg.py \
  "tests/test_gpu_parity.py::test_config4_1024_stripes_of_1mib" > $O/pytest.log 2>&1 || { echo pytest-failed; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
grep -E "graph_capture|argument_and_table|cross_stream" $O/pytest.log
