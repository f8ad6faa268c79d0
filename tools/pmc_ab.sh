#!/bin/bash
# Counters of tools/ab_bsr.py cases per library variant (abuild/<name>/, or
# "tree"), one rocprofv3 --pmc pass per counter group, each its own run:
#   tools/pmc_ab.sh TAG "VARIANTS" "CASES"
# -> gpurun_out/TAG/<variant>/<pass>/..._counter_collection.csv
# (tools/pmc_ab_summary.py TAG turns them into per-kernel means per dispatch)
set -e
TAG=$1
VARIANTS=${2:-tree}
CASES=${3:-cfg4_enc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU2"
P3="SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC"
P4="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_INPUT_VALID_READYB"
for V in $VARIANTS; do
  LIB=""
  [ "$V" = tree ] || LIB=$ROOT/abuild/$V/libzfec_hip.so
  NOCHECK=""
  [ -f "$ROOT/abuild/$V/NOCHECK" ] && NOCHECK=1  # timing-only forms: wrong bytes by design
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i + 1))
    OUT=$ROOT/gpurun_out/$TAG/$V/p$i
    mkdir -p $OUT
    ZFEC_AB_NOCHECK=$NOCHECK ZFEC_HIP_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT -o p -- \
      python3 $ROOT/tools/ab_bsr.py --worker --variants $V --cases $CASES --launches 10 > $OUT/run.log 2>&1
  done
  echo "pmc-ab $V done"
done
