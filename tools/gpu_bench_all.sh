#!/bin/bash
# GPU tests + every bench workload; each GPU step has its own limit, first failure stops.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python bench.py --cpu-seconds 5 > gpurun_out/bench_cfg2.log 2>&1
timeout -k 10 300 python bench.py --workload cfg3 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg3.log 2>&1
timeout -k 10 300 python bench.py --workload cfg4 --steps 20 --cpu-seconds 5 > gpurun_out/bench_cfg4.log 2>&1
timeout -k 10 300 python bench.py --workload cfg5 --steps 10 --cpu-seconds 5 > gpurun_out/bench_cfg5.log 2>&1
echo all-done
