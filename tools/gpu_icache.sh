#!/bin/bash
# Instruction-supply counters for the MAC kernels: list the counters the profiler offers (kept in
# counters.txt), then one PMC pass over a short bench with the instruction-cache / fetch ones
# that exist (at most 8 SQ-block counters; SQC counters in their own pass).
# usage: bash tools/gpu_icache.sh <tag>
set -e
TAG=${1:-icache}; R=$PWD; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
grep -o -E "\b(SQC_ICACHE[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_INSTS_BRANCH|SQ_INSTS_SENDMSG|SQ_WAIT_INST_ANY|SQ_INST_LEVEL[A-Z_]*|SQC_TC_INST[A-Z_]*)\b" $OUT/counters.txt | sort -u > $OUT/cands.txt || true
cat $OUT/cands.txt | tr '\n' ' '; echo
SQC=$(grep -E "^SQC_ICACHE_(HITS|MISSES|MISSES_DUPLICATE|REQ)$" $OUT/cands.txt | head -4 | tr '\n' ' ')
SQ=$(grep -E "^(SQ_IFETCH|SQ_IFETCH_LEVEL|SQ_INSTS_BRANCH|SQ_WAIT_INST_ANY)$" $OUT/cands.txt | head -4 | tr '\n' ' ')
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
if [ -n "$SQC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $SQC -f csv -d $OUT/sqc -o run -- python3 $B > $OUT/sqc.log 2>&1 || { tail -5 $OUT/sqc.log; exit 1; }
fi
if [ -n "$SQ" ]; then
  timeout -s KILL 120 rocprofv3 --pmc $SQ SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU -f csv -d $OUT/sq -o run -- python3 $B > $OUT/sq.log 2>&1 || { tail -5 $OUT/sq.log; exit 1; }
fi
python3 $R/tools/pmc_summary.py $(ls $OUT/sqc/*counter_collection.csv $OUT/sq/*counter_collection.csv 2>/dev/null) | head -60 || true
