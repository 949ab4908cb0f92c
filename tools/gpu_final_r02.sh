#!/bin/bash
# End-of-round evidence at HEAD: full GPU suite + default bench + rocprof (gpu_round.sh), per-config
# bench lines and PMC passes (gpu_pmc.sh), large-window plans, multi-rank smoke.
set -e
TAG=${1:-final}
bash tools/gpu_round.sh $TAG
bash tools/gpu_pmc.sh ${TAG}_cfg "k128r32s4096 k32r8s1024 k128r32s1500 k1024dense"
bash tools/gpu_pmc.sh ${TAG}_mixed k128r32s4096 --mixed
OUT=gpurun_out/${TAG}_large; mkdir -p $OUT
for c in "--k 256 --r 200 --m 64 --S 1504 --G 1024" "--k 128 --r 96 --m 80 --S 4096 --G 1024" "--k 512 --r 255 --m 200 --S 1504 --G 512" "--k 256 --r 200 --m 40 --S 1504 --G 1024"; do
  timeout -k 10 200 python tools/bench_large.py $c > $OUT/l.log 2>&1 || { tail -20 $OUT/l.log; exit 1; }
  tail -1 $OUT/l.log >> $OUT/large.jsonl
done
echo final done
