"""Sweep HostPipeline chunk / depth on the config-3 workload: one JSON line per setting."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from netcode_amd.pipeline import HostPipeline
    d = torch.device("cuda", 0)
    k, r, S, stride, m, G = bench.CONFIGS["k128r32s4096"]
    w = bench.Workload(d, G, k, r, S, stride, m, False, 0)
    pin = lambda t: torch.empty_like(t, device="cpu").pin_memory().copy_(t)
    h_src, h_len, h_rx, h_rxlen = pin(w.src), pin(w.src_len), pin(w.rx), pin(w.rx_len)
    h_mask, h_rmask = pin(w.smask), pin(w.rmask)
    h_rep = torch.empty((G, r, stride), dtype=torch.uint8).pin_memory()
    h_rsz = torch.empty((G, r), dtype=torch.int16).pin_memory()
    h_st = torch.empty((G, 12), dtype=torch.uint8).pin_memory()
    for chunk in (128, 256, 512, 1024):
        for depth in (2, 3, 4):
            p = HostPipeline(k, r, stride, chunk, d, depth)
            ts = []
            for _ in range(4):
                t0 = time.perf_counter()
                p.encode_decode(h_src, h_len, h_rep, h_rsz, h_rx, h_rxlen, h_mask, h_rmask, h_st,
                                w.sid, w.rid)
                torch.cuda.synchronize(d)
                ts.append(time.perf_counter() - t0)
            print(json.dumps({"chunk": chunk, "depth": depth,
                              "GiBps": round(G * k * S / min(ts[1:]) / 2**30, 2)}), flush=True)
            del p
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
