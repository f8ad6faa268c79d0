#!/bin/bash
# kernel-published completion of small synchronous calls (default) vs
# hipStreamSynchronize (ZFEC_HIP_WAIT=sync): GPU tests, then small-call latency.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
for v in sync spin sync spin; do
  echo "== ZFEC_HIP_WAIT=$v" >> gpurun_out/lat_ab2.log
  ZFEC_HIP_WAIT=$v timeout -k 10 200 python tools/bytes_latency.py >> gpurun_out/lat_ab2.log 2>&1
done
echo done
