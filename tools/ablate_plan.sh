#!/bin/bash
# Timing ablations of decode_plan_w (NTC_GF256_PLANW_ABLATE; results wrong by design, bench exits
# 3 on the failed verification): 0 none, 1 no Gauss-Jordan, 2 no D for received sources,
# 8 no decoded sizes, 11 = 1+2+8.  usage: bash tools/ablate_plan.sh <tag>
TAG=${1:-ablp}; OUT=gpurun_out/$TAG; mkdir -p $OUT
for v in 0 1 2 8 11; do
  NTC_GF256_PLANW_ABLATE=$v timeout -k 10 200 python bench.py --steps 20 --warmup 10 --no-cpu-baseline --no-host-rate > $OUT/p$v.log 2>&1
  rc=$?
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then tail -20 $OUT/p$v.log; exit 1; fi
  python -c "import json; d=json.loads(open('$OUT/p$v.log').read().strip().splitlines()[-1]); print('planw_ablate=$v', d['kernels_ms'].get('decode_plan'))"
done
