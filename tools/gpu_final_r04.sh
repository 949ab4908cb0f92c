#!/bin/bash
# End-of-round evidence at HEAD, in two gpurun calls (each under the 20-minute limit):
#   part 1: full GPU suite + default bench + rocprof kernel trace/stats + per-packet + smoke
#   part 2: per-config bench lines and PMC passes (tools/gpu_pmc.sh), mixed-m line
# usage: bash tools/gpu_final_r04.sh <tag> 1|2
set -e
TAG=${1:-r04}; PART=${2:-1}
if [ "$PART" = 1 ]; then
  bash tools/gpu_round.sh $TAG
else
  bash tools/gpu_pmc.sh ${TAG}_cfg "k128r32s4096 k32r8s1024 k128r32s1500 k1024dense"
  bash tools/gpu_pmc.sh ${TAG}_mixed k128r32s4096 --mixed
fi
echo "final part $PART done"
