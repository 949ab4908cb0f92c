#!/bin/bash
# A/B of engine variants on the GPU box: GPU parity under each variant, then bench lines per config.
# usage: bash tools/ab_mac.sh "<variant> ..." [configs...]
#   variant = "base" or comma-separated env assignments, e.g. NTC_GF256_MAC=perm,NTC_GF256_BJ_ROWS=16
set -e
mkdir -p gpurun_out
VARS=${1:-"base NTC_GF256_MAC=perm"}; shift || true
CONFS=${@:-k128r32s4096}
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate"
envof() { [ "$1" = base ] && echo "" || echo "$1" | tr ',' ' '; }
for v in $VARS; do
  tag=$(echo $v | tr ',=/.' '____')
  timeout -k 10 300 env $(envof $v) python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/par_$tag.log 2>&1 || { tail -40 gpurun_out/par_$tag.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/par_$tag.log)"
done
for c in $CONFS; do for v in $VARS; do
  tag=$(echo $v | tr ',=/.' '____')
  timeout -k 10 150 env $(envof $v) $B --config $c > gpurun_out/ab_${c}_$tag.log 2>&1
  python -c "
import json,sys; d=json.loads(open('gpurun_out/ab_${c}_$tag.log').read().strip().splitlines()[-1])
print('$c $v', d['value'], d['kernels_ms'], d['verified']['bit_exact_round_trip'], d['roofline']['byte_mac_rate_T_per_s'])"
done; done
