#!/bin/bash
# Bench-only A/B of engine variants (timing ablations included; no parity).
# usage: bash tools/ab_bench.sh "<variant> ..." [configs...]   (variant as in ab_mac.sh)
set -e
mkdir -p gpurun_out/ab
VARS=${1:-base}; shift || true
CONFS=${@:-k128r32s4096}
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate"
envof() { [ "$1" = base ] && echo "" || echo "$1" | tr ',' ' '; }
for c in $CONFS; do for v in $VARS; do
  tag=$(echo $v | tr ',=/.' '____')
  rc=0; timeout -k 10 150 env $(envof $v) $B --config $c > gpurun_out/ab/${c}_$tag.log 2>&1 || rc=$?
  # a timing ablation fails verification (rc 3) but still prints its line; anything else stops
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -5 gpurun_out/ab/${c}_$tag.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/ab/${c}_$tag.log').read().strip().splitlines()[-1])
print('$c $v', d['value'], d['kernels_ms'], d['verified']['bit_exact_round_trip'])"
done; done
