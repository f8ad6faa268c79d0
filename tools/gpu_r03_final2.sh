#!/bin/bash
# Round-3 closing session, part A: the full GPU suite, smoke, a bench line of
# every workload (cfg2 with the CPU baseline), the bytes-API latencies and the
# host cost per call, and the K=20/M=60 memory-pattern probe.  Every GPU step
# has its own time limit; the first failure ends the script.
# usage: tools/gpu_r03_final2.sh TAG     (part B: bash tools/profile_r02.sh TAGprof cfg2 cfg3 cfg4 cfg5)
set -e
export TMPDIR=/tmp
T=${1:-r03z}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/$T/bench_cfg2.log 2>&1
for W in cfg3 cfg4 cfg5; do
  timeout -k 10 400 python bench.py --workload $W --steps 20 --warmup 3 --no-cpu > gpurun_out/$T/bench_$W.log 2>&1
done
timeout -k 10 300 python tools/bytes_latency.py > gpurun_out/$T/bytes_latency.log 2>&1
timeout -k 10 120 ./tools/host_cost.exe > gpurun_out/$T/host_cost.log 2>&1
timeout -k 10 200 ./tools/mb_pattern.exe 10 > gpurun_out/$T/mb_pattern.log 2>&1
echo done
