#!/bin/bash
# Round-3 measurement session: bench lines of every workload (cfg2 with the CPU baseline),
# the rocprofv3 leg profiles (kernel trace + FETCH_SIZE + WRITE_SIZE passes), the bytes-API
# latencies.  Every GPU step under its own limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
T=${1:-r03f}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/${T}_bench_cfg2.log 2>&1
for W in cfg3 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_bench_$W.log 2>&1
done
bash tools/profile_r02.sh ${T}prof cfg2 cfg3 cfg4 cfg5 > gpurun_out/${T}_profile.log 2>&1
timeout -k 10 300 python tools/bytes_latency.py > gpurun_out/${T}_bytes_latency.log 2>&1
timeout -k 10 300 python tools/wide_bench.py --variants shipped > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.log
echo done
