#!/bin/bash
# Per-config evidence: the full bench line (roofline + CPU baseline), then the rocprofv3 PMC
# passes bench.py reads back (FETCH_SIZE, WRITE_SIZE, two SQ passes), each its own profiler run.
# usage: bash tools/gpu_pmc.sh <tag> "<config> [<config> ...]" [--mixed]
set -e
TAG=${1:-pmc}; CFGS=${2:-k128r32s4096}; EXTRA=${3:-}
R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for C in $CFGS; do
  timeout -k 10 400 python $R/bench.py --config $C $EXTRA > $OUT/bench_$C.log 2>&1 || { tail -20 $OUT/bench_$C.log; exit 1; }
  echo "$C: $(grep '^{' $OUT/bench_$C.log | cut -c1-160)"
  [ -n "$EXTRA" ] && continue
  B="$R/bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
  (cd /tmp
   timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/$C/fetch -o run -- python3 $B > $OUT/$C.fetch.log 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/$C/write -o run -- python3 $B > $OUT/$C.write.log 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU -f csv -d $OUT/$C/sq -o run -- python3 $B > $OUT/$C.sq.log 2>&1 &&
   timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $OUT/$C/sq2 -o run -- python3 $B > $OUT/$C.sq2.log 2>&1) || { echo "pmc passes of $C failed"; tail -5 $OUT/$C.*.log; exit 1; }
  echo "$C: pmc passes done"
done
