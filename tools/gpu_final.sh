#!/bin/bash
# End-of-session evidence: GPU suite, smoke, default bench line, rocprof kernel stats, PMC traffic
# passes, torchrun N=1 bench path.   usage: bash tools/gpu_final.sh <tag>
set -e
TAG=${1:-final}
bash tools/gpu_round.sh $TAG
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
bash tools/gpu_profile.sh ${TAG}_prof
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/$TAG/torchrun1.log 2>&1
tail -1 gpurun_out/$TAG/torchrun1.log
