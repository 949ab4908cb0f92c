#!/bin/bash
# Lean-loop MAC (default for full 2 KiB spans; NTC_BJ_FULL=0 = the general loop): parity suites,
# then interleaved bench lines for config 3 (x2) and config 5.  usage: bash tools/ab_full.sh <tag>
set -e
TAG=${1:-full}; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_capi.py tests/test_gpu_pipeline.py tests/test_gpu_dense.py tests/test_gpu_large_window.py -x -q --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
echo "parity: $(tail -1 $OUT/parity.log)"
run() {  # tag env-value extra-args
  NTC_BJ_FULL=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate $3 > $OUT/$1_f$2.log 2>&1 || { tail -20 $OUT/$1_f$2.log; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/$1_f$2.log').read().strip().splitlines()[-1]); print('$1 full=$2', d['value'], d['kernels_ms'])"
}
for rep in 1 2; do run c3_$rep 1 ""; run c3_$rep 0 ""; done
run mixed 1 "--mixed"; run mixed 0 "--mixed"
run c5 1 "--config k1024dense"; run c5 0 "--config k1024dense"
