#!/bin/bash
# A/B of the in-tree libntc_gf256.so against another build (NTC_GF256_LIB=<path>): bench lines
# interleaved, 3 rounds.  usage: bash tools/ab_lib.sh <other .so> [bench args]
set -e
OTHER=$1; shift
OUT=gpurun_out/ab_lib; mkdir -p $OUT
for rep in 1 2 3; do
  for v in cur other; do
    if [ $v = other ]; then export NTC_GF256_LIB=$OTHER; else unset NTC_GF256_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate "$@" > $OUT/${v}_$rep.log 2>&1 || { tail -20 $OUT/${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$OUT/${v}_$rep.log') if l.startswith('{')][-1]); print('$v:', d['value'], d['ms_per_step'], d['kernels_ms'])"
  done
done
