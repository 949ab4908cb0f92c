#!/bin/bash
# SQ counters (wave time split) for the bench's kernels.  usage: bash tools/gpu_sq.sh <tag> [extra env]
set -e
TAG=${1:-sq}; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU -f csv -d $OUT/sq -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate > $OUT/sq2.log 2>&1 || { tail -20 $OUT/sq2.log; exit 1; }
echo done
