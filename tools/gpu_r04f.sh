set -e
R=$PWD; OUT=$R/gpurun_out/r04f; mkdir -p $OUT
export TMPDIR=/tmp
NTC_GF256_LIB=exp/libntc_gf256_dnclk.so timeout -k 10 120 python tools/dense_clock.py > $OUT/dense_clock.json
cut -c1-1500 $OUT/dense_clock.json
(cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/dtrace -o run -- python3 $R/tools/dense_invert_time.py --iters 5 > $OUT/dtrace.log 2>&1) || { tail -5 $OUT/dtrace.log; exit 1; }
find $OUT/dtrace -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -12
B="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-host-rate"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -f csv -d $OUT/plan_pmc -o run -- python3 $B > $OUT/plan_pmc.log 2>&1) || { echo "pmc pass failed"; tail -5 $OUT/plan_pmc.log; }
find $OUT/plan_pmc -name "*counter_collection.csv" | head -2
