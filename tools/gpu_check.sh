#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench, and a kernel-trace profile.
# Every GPU step has its own time limit; the first failure ends the script.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 8 > gpurun_out/bench.log 2>&1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
echo done
