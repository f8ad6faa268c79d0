#!/bin/bash
# Counter passes over tools/jit_probe.py (K=20/M=60 encode: real kernel, all-zero data,
# no-HBM and no-arithmetic probes), one rocprofv3 run per pass, each under its own limit:
#   tools/jit_probe_pmc.sh TAG [SHAPE VARIANTS]   (SHAPE: cfg4 (default) or cfg3)
# Effective clock per dispatch = GRBM_GUI_ACTIVE / 8 / kernel time (MI355X_MICROARCH.md,
# DVFS give-back); HBM bytes = 2 * FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE halving).
set -e
TAG=${1:-probe}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
OUT=$ROOT/gpurun_out/$TAG
mkdir -p $OUT
ARGS="--rounds 2 --reps 30 --warm 30 --shape ${2:-cfg4} --variants ${3:-real,zero,nohbm,noarith}"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES --output-format csv -d $OUT/clk -o clk -- python3 $ROOT/tools/jit_probe.py $ARGS --legs-out $OUT/clk_legs.json > $OUT/clk.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $ROOT/tools/jit_probe.py $ARGS --legs-out $OUT/fetch_legs.json > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $ROOT/tools/jit_probe.py $ARGS --legs-out $OUT/write_legs.json > $OUT/write.log 2>&1
echo jit-probe-pmc-done
