#!/bin/bash
# Clock-ramp experiment: bench value at the driver's --steps 20 --warmup 5 with and without a
# longer HBM copy probe ahead of the warmup, against --warmup 30; twice each, interleaved.
set -e
OUT=gpurun_out/warm; mkdir -p $OUT
for rep in 1 2; do
  for v in "5 0" "5 200" "30 0"; do
    set -- $v
    NTC_BENCH_PROBE_FIRST=$2 timeout -k 10 300 python bench.py --steps 20 --warmup $1 --no-cpu-baseline --no-host-rate > $OUT/w$1_p$2_$rep.log 2>&1 || { tail -20 $OUT/w$1_p$2_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$OUT/w$1_p$2_$rep.log') if l.startswith('{')][-1]); print('warmup $1 probe $2:', d['value'], d['roofline']['kernel_ms'], d['roofline']['hbm_copy_probe_GBps'])"
  done
done
