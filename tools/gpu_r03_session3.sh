#!/bin/bash
# Round-3 session 3: grouped matapply_bsg launches -- bit-sliced parity tests, the wide-code
# bench, the default bench (host enqueue figure).
set -e
export TMPDIR=/tmp
T=${1:-r03s3}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bsg.py tests/test_gpu_jit.py tests/test_gpu_parity.py -x -q -m gpu -k "bsg or jit or small_launch or ragged or wide" --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
timeout -k 10 400 python tools/wide_bench.py --variants shipped > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.err
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --no-extra > gpurun_out/${T}_bench_cfg2.log 2>&1
echo done
