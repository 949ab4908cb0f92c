#!/bin/bash
# A/B of two environments on the same tree: bench lines interleaved, 3 rounds.
# usage: bash tools/ab_env.sh "<env A>" "<env B>" [bench args]   e.g. "" "NTC_GF256_MAC=solo"
set -e
A=$1; B=$2; shift 2
OUT=gpurun_out/ab_env; mkdir -p $OUT
for rep in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then E=$A; else E=$B; fi
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-rate "$@" > $OUT/${v}_$rep.log 2>&1 || { tail -20 $OUT/${v}_$rep.log; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$OUT/${v}_$rep.log') if l.startswith('{')][-1]); print('$v [$E]:', d['value'], d['ms_per_step'], d['kernels_ms'])"
  done
done
