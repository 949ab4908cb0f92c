"""Time the dense inversion (config-5 shape) alone: ntc_gf256_dense_invert_batch on a random
n x n matrix, mean over --iters launches (HIP events on the engine's stream).
usage: python tools/dense_invert_time.py [--n 1024] [--G 1] [--iters 20]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netcode_amd.engine import DenseCode  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--G", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    g = torch.Generator().manual_seed(5)
    mat = torch.randint(0, 256, (a.G, a.n, a.n), dtype=torch.uint8, generator=g).cuda()
    dc = DenseCode(0)
    for _ in range(3):
        dc.invert(mat)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(a.iters):
        inv, ok = dc.invert(mat)
    t1.record()
    torch.cuda.synchronize()
    print(json.dumps({"n": a.n, "G": a.G, "invert_ms": round(t0.elapsed_time(t1) / a.iters, 4),
                      "ok": int(ok.sum())}))


if __name__ == "__main__":
    main()
