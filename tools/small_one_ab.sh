#!/bin/bash
# A/B of the small synchronous call's kernel: matapply_one (default) against
# matapply_reg (ZFEC_HIP_SMALL_ONE=0), interleaved rounds on one box: kernel
# trace of 2000 x 4 KiB K=3/M=10 encodes + decodes from bytes, and the bytes
# API latency.  usage: tools/small_one_ab.sh TAG
set -e
export TMPDIR=/tmp
T=${1:-one_ab}
mkdir -p gpurun_out/$T
for round in 1 2; do
  for v in 1 0; do
    ZFEC_HIP_SMALL_ONE=$v N=2000 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$T -o r${round}_one$v -- python tools/small_call_probe.py 3,10,4096 > gpurun_out/$T/r${round}_one$v.log 2>&1
    ZFEC_HIP_SMALL_ONE=$v N=5000 timeout -k 10 200 python tools/small_call_probe.py 3,10,4096 5,9,4096 > gpurun_out/$T/lat_r${round}_one$v.log 2>&1
  done
done
echo done
