#!/bin/bash
# GPU session: parity tests (incl. the bit-sliced JIT kernels), JIT A/B, benches.
# Each GPU step has its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo pytest-ok
timeout -k 10 400 python -u tools/jit_bench.py > gpurun_out/jit_bench.log 2>&1
echo jitbench-ok
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_cfg2.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 20 --no-cpu > gpurun_out/bench_cfg3.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 --no-cpu > gpurun_out/bench_cfg4.log 2>&1
echo all-done
