#!/bin/bash
# Round-3 session 2: launch-API host cost, K=20/M=60 residency caps, benches with the
# settled-clock back-to-back legs, wide codes (k > 32) against round 2's passes.
set -e
export TMPDIR=/tmp
T=${1:-r03s2}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/host_cost.exe > gpurun_out/${T}_host_cost.log 2>&1
timeout -k 10 240 python tools/jit_probe.py --rounds 2 --variants real,lds2,lds1,noarith > gpurun_out/${T}_jit_probe.json 2> gpurun_out/${T}_jit_probe.err
timeout -k 10 300 python bench.py --workload cfg4 --steps 20 --warmup 3 --no-cpu > gpurun_out/${T}_bench_cfg4.log 2>&1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > gpurun_out/${T}_bench_cfg2.log 2>&1
timeout -k 10 400 python tools/wide_bench.py > gpurun_out/${T}_wide.json 2> gpurun_out/${T}_wide.err
echo done
