#!/bin/bash
# Full GPU check after a kernel change: parity tests, every bench workload, rocprofv3 passes.
set -e
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
TAG=${1:-prof}
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo pytest-ok
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_cfg2.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg3.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg4.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --cpu-seconds 5 > gpurun_out/bench_cfg5.log 2>&1
echo benches-ok
bash tools/profile_round.sh $TAG cfg2 cfg3 cfg4 cfg5
