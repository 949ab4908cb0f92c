#!/bin/bash
# Quick GPU check of the current tree: parity suites, then bench lines for configs 3 (x2), 3 mixed,
# 2, 4 and 5.  usage: bash tools/gpu_check.sh <tag>
set -e
TAG=${1:-check}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_window.py tests/test_gpu_capi.py tests/test_gpu_pipeline.py tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
echo "parity: $(tail -1 $OUT/parity.log)"
run() {  # tag extra-args
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate $2 > $OUT/$1.log 2>&1 || { tail -20 $OUT/$1.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['kernels_ms'])"
}
run c3a ""; run c3b ""; run mixed "--mixed"; run c2 "--config k32r8s1024"; run c4 "--config k128r32s1500"; run c5 "--config k1024dense"
