#!/bin/bash
# A/B of the shared-table bit-sliced chains (NTC_GF256_BJ_GX=1|2) against the nibble chain (0):
# parity suites under each variant, then the default bench line for each, interleaved twice.
# usage: bash tools/ab_gx.sh <tag> [variants to test, default "1 2"]
set -e
TAG=${1:-gx}; VARS=${2:-"1 2"}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in $VARS; do
  NTC_GF256_BJ_GX=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_window.py -x -q --timeout 300 --timeout-method thread > $OUT/parity_gx$v.log 2>&1 || { tail -30 $OUT/parity_gx$v.log; exit 1; }
  echo "parity gx=$v: $(tail -1 $OUT/parity_gx$v.log)"
done
for rep in 1 2; do
  for v in 0 $VARS; do
    NTC_GF256_BJ_GX=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_gx${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_gx${v}_$rep.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/bench_gx${v}_$rep.log').read().strip().splitlines()[-1]); print('gx=$v', d['value'], d['kernels_ms'])"
  done
done
