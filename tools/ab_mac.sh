#!/bin/bash
# A/B of MAC variants on the GPU box: parity under the variant, then bench lines per config.
# usage: bash tools/ab_mac.sh "<variants>" [configs...]
set -e
mkdir -p gpurun_out
VARS=${1:-"perm bitslice"}; shift || true
CONFS=${@:-k128r32s4096}
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-rate"
for v in $VARS; do
  [ "$v" = perm ] && continue
  timeout -k 10 300 env NTC_GF256_MAC=$v python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/par_bs$v.log 2>&1 || { tail -40 gpurun_out/par_bs$v.log; exit 1; }
  echo "parity bs=$v: $(tail -1 gpurun_out/par_bs$v.log)"
done
for c in $CONFS; do for v in $VARS; do
  timeout -k 10 150 env NTC_GF256_MAC=$v $B --config $c > gpurun_out/ab_${c}_$v.log 2>&1
  python -c "
import json,sys; d=json.loads(open('gpurun_out/ab_${c}_$v.log').read().strip().splitlines()[-1])
print('$c bs=$v', d['value'], d['kernels_ms'], d['verified'], d['roofline']['byte_mac_rate_T_per_s'])"
done; done
