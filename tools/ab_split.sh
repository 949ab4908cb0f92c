#!/bin/bash
# A/B of the split batches (NTC_GF256_SPLIT=1 default vs 0): bench lines interleaved, 3 rounds.
set -e
OUT=gpurun_out/ab_split; mkdir -p $OUT
for rep in 1 2 3; do
  for v in 1 0; do
    NTC_GF256_SPLIT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/s${v}_$rep.log 2>&1 || { tail -20 $OUT/s${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$OUT/s${v}_$rep.log') if l.startswith('{')][-1]); print('split $v:', d['value'], d['ms_per_step'], d['kernels_ms'])"
  done
done
