#!/bin/bash
# Variant-4 chain: GPU parity suites under the default (variant 4 where the probe allows it), then
# bench lines of variant 4 against variant 3 (NTC_GF256_BJ_GX=3), interleaved; dense bench with
# the row-tile-fastest task order against the column-span-fastest one.
# usage: bash tools/ab_gx4.sh <tag>
set -e
TAG=${1:-gx4}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_window.py tests/test_gpu_capi.py tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
echo "parity: $(tail -1 $OUT/parity.log)"
for rep in 1 2; do
  for v in 4 3; do
    NTC_GF256_BJ_GX=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate > $OUT/bench_gx${v}_$rep.log 2>&1 || { tail -20 $OUT/bench_gx${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_gx${v}_$rep.log').read().strip().splitlines()[-1]); print('gx=$v', d['value'], d['kernels_ms'])"
  done
done
for v in tile cc; do
  NTC_BJ_ORDER=$v timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline --no-host-rate > $OUT/dense_$v.log 2>&1 || { tail -20 $OUT/dense_$v.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/dense_$v.log').read().strip().splitlines()[-1]); print('order=$v', d['value'], d['kernels_ms'])"
done
