#!/bin/bash
# A/B of the shared-table bit-sliced chain (NTC_GF256_BJ_GX=1) against the nibble chain: parity
# suite under the variant, then the default bench line for each (same box, back to back).
# usage: bash tools/ab_gx.sh <tag>
set -e
TAG=${1:-gx}; OUT=gpurun_out/$TAG; mkdir -p $OUT
NTC_GF256_BJ_GX=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_window.py -x -q --timeout 300 --timeout-method thread > $OUT/parity_gx.log 2>&1 || { tail -30 $OUT/parity_gx.log; exit 1; }
tail -1 $OUT/parity_gx.log
for v in 0 1 0 1; do
  NTC_GF256_BJ_GX=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_gx$v.log 2>&1 || { tail -20 $OUT/bench_gx$v.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_gx$v.log').read().strip().splitlines()[-1]); print('gx=$v', d['value'], d['kernels_ms'])"
done
