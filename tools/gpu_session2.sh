#!/bin/bash
# Benches of every workload + rocprofv3 kernel trace / FETCH_SIZE / WRITE_SIZE passes.
set -e
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/bench_cfg2.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg3 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg3.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg4.log 2>&1
timeout -k 10 300 python -u bench.py --workload cfg5 --steps 10 --cpu-seconds 5 > gpurun_out/bench_cfg5.log 2>&1
echo benches-ok
bash tools/profile_round.sh prof_r01d cfg2 cfg3 cfg4 cfg5
