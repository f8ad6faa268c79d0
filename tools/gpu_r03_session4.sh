#!/bin/bash
# Round-3 session 4: 94/100 on the bit-sliced JIT with row tiles of 10 / 3 / 2 / 1 rows
# (ZFEC_HIP_JIT_TILE; more, shorter tiles = more waves per unit, each loading every input).
set -e
export TMPDIR=/tmp
T=${1:-r03s4}
mkdir -p gpurun_out
for t in 10 3 2 1; do
  ZFEC_HIP_JIT_TILE=$t timeout -k 10 200 python tools/wide_bench.py --shapes 94/100 --variants shipped > gpurun_out/${T}_wide_t$t.json 2> gpurun_out/${T}_wide_t$t.err
done
echo done
