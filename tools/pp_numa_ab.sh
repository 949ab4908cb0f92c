#!/bin/bash
# Per-packet C driver, pinned pool slabs placed next to the GPU (NTC_BATCH_PINNED_NUMA=gpu) vs next to the calling
# thread (default: hipHostRegister on malloc pages), interleaved; prints encode / decode seconds.
# usage: bash tools/pp_numa_ab.sh [reps]
set -o pipefail
REPS=${1:-3}; OUT=gpurun_out/pp_numa; mkdir -p $OUT
for rep in $(seq $REPS); do
  for v in gpu local; do
    for M in batched async; do
      if [ $v = gpu ]; then export NTC_BATCH_PINNED_NUMA=gpu; else unset NTC_BATCH_PINNED_NUMA; fi
      timeout -k 10 120 tests/_build/pp_driver $M 256 128 1024 32 4 10 7 > $OUT/${v}_${M}_$rep.log 2>&1 || { tail -5 $OUT/${v}_${M}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${v}_${M}_$rep.log').read().strip().splitlines()[-1]); print('$v $M', d['encode_s'], d['decode_s'], d['encode_s'] + d['decode_s'], d['packets_hash'], d['deliveries_hash'])"
    done
  done
done
