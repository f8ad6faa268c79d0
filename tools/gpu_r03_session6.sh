#!/bin/bash
# Round-3 session 6: matapply_bsg row-group target (workgroups per CU) on the wide codes.
set -e
export TMPDIR=/tmp
T=${1:-r03s6}
mkdir -p gpurun_out
for w in 1 2 4 8; do
  ZFEC_HIP_BSG_WGS=$w timeout -k 10 200 python tools/wide_bench.py --shapes 128/256,200/256 --variants shipped > gpurun_out/${T}_wide_w$w.json 2> gpurun_out/${T}_wide_w$w.err
done
echo done
