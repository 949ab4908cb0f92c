#!/bin/bash
# GF(2^w) combine: parity (tests/test_gpu_gfw.py), then tools/bench_gfw.py interleaved against
# another libntc_gf256.so build (NTC_GF256_LIB).  usage: bash tools/gpu_gfw_ab.sh <tag> <other .so>
set -o pipefail
TAG=$1; OTHER=$2; OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gfw.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/gfw_tests.log 2>&1 || { tail -20 $OUT/gfw_tests.log; exit 1; }
tail -1 $OUT/gfw_tests.log
for rep in 1 2; do
  timeout -k 10 120 python tools/bench_gfw.py > $OUT/cur_$rep.json 2>&1 || { tail -5 $OUT/cur_$rep.json; exit 1; }
  echo "cur: $(tail -1 $OUT/cur_$rep.json | cut -c1-400)"
  NTC_GF256_LIB=$OTHER timeout -k 10 120 python tools/bench_gfw.py > $OUT/other_$rep.json 2>&1 || { tail -5 $OUT/other_$rep.json; exit 1; }
  echo "other: $(tail -1 $OUT/other_$rep.json | cut -c1-400)"
done
