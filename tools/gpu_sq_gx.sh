#!/bin/bash
# SQ counter passes of the bench's MAC kernels under a given environment (A/B of chain variants).
# usage: bash tools/gpu_sq_gx.sh <tag> <NTC_GF256_BJ_GX value>
set -e
TAG=${1:-sqgx}; GX=${2:-1}; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp NTC_GF256_BJ_GX=$GX
cd /tmp
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU -f csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/sq2 -o run -- python3 $B > $OUT/sq2.log 2>&1 || { tail -20 $OUT/sq2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_FLAT GRBM_COUNT GRBM_GUI_ACTIVE -f csv -d $OUT/sq3 -o run -- python3 $B > $OUT/sq3.log 2>&1 || { tail -20 $OUT/sq3.log; echo "sq3 failed (counter names?)"; }
echo done
