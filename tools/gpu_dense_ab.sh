#!/bin/bash
# Dense (config 5) panel A/B: the dense parity suite under the default panel kernel, then the
# k1024dense bench line under the default and under NTC_DENSE_PANEL=own, interleaved (ra = the default run-ahead panel).
# usage: bash tools/gpu_dense_ab.sh <tag>
set -e
TAG=${1:-dense}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $OUT/dense_tests.log 2>&1 || { tail -30 $OUT/dense_tests.log; exit 1; }
echo "dense parity: $(tail -1 $OUT/dense_tests.log)"
for rep in 1 2; do
  for v in ra own; do
    NTC_DENSE_PANEL=$v timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline --no-host-rate > $OUT/bench_${v}_${rep}.log 2>&1 || { tail -20 $OUT/bench_${v}_${rep}.log; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/bench_${v}_${rep}.log').read().strip().splitlines()[-1]); print('panel=$v', d['value'], d['kernels_ms'])"
  done
done
