#!/bin/bash
# SQ counters of one general-kernel variant on one shape (tools/mb_encode.exe MB_AB mode).
# usage: tools/counters_gen.sh <k,r> <variant> <tag>
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cnt_$3
cd /tmp
export MB_AB=1 MB_SHAPE=$1 MB_VARIANT=$2
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/cnt_$3/kt -o run -- $R/tools/mb_encode.exe > $R/gpurun_out/cnt_$3/kt.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES -f csv -d $R/gpurun_out/cnt_$3/p1 -o run -- $R/tools/mb_encode.exe > $R/gpurun_out/cnt_$3/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -f csv -d $R/gpurun_out/cnt_$3/p2 -o run -- $R/tools/mb_encode.exe > $R/gpurun_out/cnt_$3/p2.log 2>&1
echo ok
