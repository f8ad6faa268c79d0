#!/bin/bash
# Round-3 check session: parity tests, smoke, the default bench and the wide-code bench.
# Every GPU step has its own time limit; the first failure ends the script.
# usage: tools/gpu_r03_check.sh TAG [pytest -k expression]
set -e
export TMPDIR=/tmp
TAG=${1:-check}
mkdir -p gpurun_out
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "$2" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 120 ./tools/host_cost.exe > gpurun_out/${TAG}_host_cost.log 2>&1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/${TAG}_bench_cfg2.log 2>&1
timeout -k 10 300 python bench.py --workload cfg4 --steps 20 --warmup 3 --no-cpu > gpurun_out/${TAG}_bench_cfg4.log 2>&1
echo done
