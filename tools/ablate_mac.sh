#!/bin/bash
# Timing ablations of the encode MAC (NTC_GF256_BJ_ABLATE, results deliberately wrong; bench exits
# 3 on the failed verification, which is expected here).  Prints encode MAC ms per ablation.
# usage: bash tools/ablate_mac.sh <tag> ["0 1 2 3 16 64 67"]
TAG=${1:-abl}; VARS=${2:-"0 1 2 3 16 64 67"}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for rep in 1 2; do
  for v in $VARS; do
    NTC_GF256_BJ_ABLATE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-rate > $OUT/abl${v}_$rep.log 2>&1
    rc=$?
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -20 $OUT/abl${v}_$rep.log; exit 1; fi
    python -c "import json; d=json.loads(open('$OUT/abl${v}_$rep.log').read().strip().splitlines()[-1]); print('abl=$v', d['kernels_ms'].get('encode_mac'), d['kernels_ms'].get('decode_mac'))"
  done
done
