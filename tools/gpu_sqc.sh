#!/bin/bash
# Two SQ PMC passes of one config (instruction cache, branches, SALU and wait attribution);
# usage: bash tools/gpu_sqc.sh <tag> [config]
set -e
TAG=$1; C=${2:-k128r32s4096}
R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
B="$R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY -f csv -d $OUT/sqc1 -o run -- python3 $B > $OUT/sqc1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/sqc2 -o run -- python3 $B > $OUT/sqc2.log 2>&1
echo "sqc passes done"
