"""Per-step wall times of the config-3 step from a cold start (each step synchronised), to see how
many steps the device needs to reach its steady rate; optional pre-load (--preload matmul|copy).
usage: python tools/step_times.py [--steps 40] [--preload none|matmul|copy]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--preload", default="none")
a = ap.parse_args()
dev = torch.device("cuda", 0)
k, r, S, stride, m, G = bench.CONFIGS["k128r32s4096"]
w = bench.Workload(dev, G, k, r, S, stride, m, False, 0)
torch.cuda.synchronize(dev)
if a.preload == "matmul":
    x = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        y = x @ x
    torch.cuda.synchronize(dev)
elif a.preload == "copy":
    bench.hbm_copy_probe(dev, reps=200)
ts = []
for _ in range(a.steps):
    t0 = time.perf_counter()
    w.step()
    torch.cuda.synchronize(dev)
    ts.append(round((time.perf_counter() - t0) * 1e3, 3))
print(json.dumps({"preload": a.preload, "ms": ts}))
