#!/bin/bash
# A/B of the small synchronous call's input path: matapply_one with the inputs
# in its argument block (default), from the bounce buffer over PCIe
# (ZFEC_HIP_SMALL_INLINE=0), and matapply_reg (ZFEC_HIP_SMALL_ONE=0);
# interleaved rounds on one box, bytes-API latency (5000 calls each) and a
# kernel trace per variant.  usage: tools/small_inline_ab.sh TAG
set -e
export TMPDIR=/tmp
T=${1:-inline_ab}
mkdir -p gpurun_out/$T
for round in 1 2 3; do
  for v in "inline" "pinned" "reg"; do
    case $v in
      inline) E="";;
      pinned) E="ZFEC_HIP_SMALL_INLINE=0";;
      reg) E="ZFEC_HIP_SMALL_ONE=0";;
    esac
    env $E N=5000 timeout -k 10 200 python tools/small_call_probe.py 3,10,4096 2,4,4096 > gpurun_out/$T/lat_r${round}_$v.log 2>&1
  done
done
for v in "inline" "pinned"; do
  case $v in
    inline) E="";;
    pinned) E="ZFEC_HIP_SMALL_INLINE=0";;
  esac
  env $E N=2000 timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$T -o kt_$v -- python tools/small_call_probe.py 3,10,4096 > gpurun_out/$T/kt_$v.log 2>&1
done
echo done
