#!/bin/bash
# Dense parity suite, then config-5 bench lines.  usage: bash tools/gpu_dense_check.sh <tag>
set -e
TAG=${1:-dense}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $OUT/dense_tests.log 2>&1 || { tail -30 $OUT/dense_tests.log; exit 1; }
echo "dense parity: $(tail -1 $OUT/dense_tests.log)"
for rep in 1 2; do
  timeout -k 10 300 python bench.py --config k1024dense --no-cpu-baseline --no-host-rate > $OUT/c5_$rep.log 2>&1 || { tail -20 $OUT/c5_$rep.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c5_$rep.log').read().strip().splitlines()[-1]); print('c5', d['value'], d['kernels_ms'])"
done
