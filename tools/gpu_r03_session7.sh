#!/bin/bash
# fec_run_batch_jobs / matapply_pair: GPU tests, then the cfg2 step as one paired
# launch (both workgroup orders) against the default 2-stream eager step, interleaved.
set -e
export TMPDIR=/tmp
T=${1:-r03s7}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_batch_jobs.py > gpurun_out/${T}_tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu --no-extra > gpurun_out/${T}_streams2_$rep.json 2> gpurun_out/${T}_err.log
  ZFEC_HIP_PAIR_ORDER=0 timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu --no-extra --paired > gpurun_out/${T}_pair0_$rep.json 2>> gpurun_out/${T}_err.log
  ZFEC_HIP_PAIR_ORDER=1 timeout -k 10 200 python bench.py --steps 200 --warmup 5 --no-cpu --no-extra --paired > gpurun_out/${T}_pair1_$rep.json 2>> gpurun_out/${T}_err.log
done
echo done
