#!/bin/bash
# Batch-adaptor tests against the in-tree libraries, then (on this scratch copy only) with
# libntc_gf256.so swapped for another build: usage: bash tools/gpu_gather_ab.sh <tag> <other .so>
set -o pipefail
TAG=$1; OTHER=$2; OUT=gpurun_out/$TAG; mkdir -p $OUT
T="tests/test_gpu_gather.py tests/test_gpu_batch.py tests/test_gpu_capi.py"
timeout -k 10 300 python -u -m pytest $T -q -m gpu --timeout 120 --timeout-method thread > $OUT/cur.log 2>&1
rc=$?; tail -4 $OUT/cur.log; echo "cur rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
cp "$OTHER" netcode_amd/libntc_gf256.so
timeout -k 10 300 python -u -m pytest $T -q -m gpu --timeout 120 --timeout-method thread > $OUT/other.log 2>&1
rc=$?; tail -4 $OUT/other.log; echo "other rc=$rc"
