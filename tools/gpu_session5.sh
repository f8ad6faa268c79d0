#!/bin/bash
# flag wait (default) vs hipStreamSynchronize (ZFEC_HIP_WAIT=sync): GPU tests,
# the sync probe, small-call latency of the bytes API, and the default bench.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 90 tools/mb_sync.exe > gpurun_out/sync.log 2>&1
for v in sync spin sync spin; do
  echo "== ZFEC_HIP_WAIT=$v" >> gpurun_out/lat_ab.log
  ZFEC_HIP_WAIT=$v timeout -k 10 200 python tools/bytes_latency.py >> gpurun_out/lat_ab.log 2>&1
done
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_wait.json 2>&1
echo done
