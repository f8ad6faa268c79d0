#!/bin/bash
# Round-3 baseline session on the GPU box: parity tests, smoke and the default bench
# on the round-2 tree.  Every GPU step has its own time limit; the first failure ends it.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03_base_pytest.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_base_smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/r03_base_bench.log 2>&1
echo done
