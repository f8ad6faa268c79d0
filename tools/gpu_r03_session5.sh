#!/bin/bash
# Round-3 session 5: full GPU suite on the current tree, wide codes, the default benches.
set -e
export TMPDIR=/tmp
T=${1:-r03s5}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
timeout -k 10 400 python tools/wide_bench.py > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.err
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/${T}_bench_cfg2.log 2>&1
timeout -k 10 300 python bench.py --workload cfg4 --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_bench_cfg4.log 2>&1
echo done
