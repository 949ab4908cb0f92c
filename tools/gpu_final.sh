set -e
bash tools/gpu_round.sh s5final
bash tools/gpu_profile.sh s5prof
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 > gpurun_out/s5final/torchrun1.log 2>&1
tail -1 gpurun_out/s5final/torchrun1.log
