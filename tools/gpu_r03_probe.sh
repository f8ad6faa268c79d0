#!/bin/bash
# Round-3 probe session: host launch cost by kernel-argument size, the K=20/M=60 JIT
# probes timed (tools/jit_probe.py) and under counters (tools/jit_probe_pmc.sh).
set -e
export TMPDIR=/tmp
TAG=${1:-probe}
mkdir -p gpurun_out
timeout -k 10 120 ./tools/host_cost.exe > gpurun_out/${TAG}_host_cost.log 2>&1
timeout -k 10 240 python tools/jit_probe.py --rounds 3 > gpurun_out/${TAG}_jit_probe.json 2> gpurun_out/${TAG}_jit_probe.err
bash tools/jit_probe_pmc.sh ${TAG}_pmc
echo done
