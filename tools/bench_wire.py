"""Throughput of the device wire-format kernels (ntc_gf256_write_repairs / write_sources /
read_packets) at the config-3 shape (k=128 r=32 4 KiB, G=4096), timed with HIP events on the
engine's stream; prints one JSON line.  Algorithmic bytes per launch = bytes read + bytes written
(payload copies; header/id bytes included), against the 8 TB/s HBM peak.

usage: python tools/bench_wire.py [--G 4096] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps, stream):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record(stream)
    for _ in range(reps):
        fn()
    ev[1].record(stream)
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    from netcode_amd import BatchEncoder, Wire
    dev = torch.device("cuda", 0)
    G, k, r, S = a.G, 128, 32, 4096
    g = torch.Generator(device=dev).manual_seed(3)
    src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=g)
    lens = torch.full((G, k), S, dtype=torch.int16, device=dev)
    enc = BatchEncoder(k, r, dev)(src, lens)
    w = Wire(dev)
    s = torch.cuda.current_stream(dev)
    out = {}
    rp, rl = w.write_repairs(enc, k)
    t = timed(lambda: w.write_repairs(enc, k), a.reps, s)
    nbytes = G * r * S + int(rl.sum().item())
    out["write_repairs"] = {"ms": round(t, 4), "GBps": round(nbytes / t / 1e6, 1),
                            "bytes_per_launch": nbytes}
    sp, sl = w.write_sources(src, lens)
    t = timed(lambda: w.write_sources(src, lens), a.reps, s)
    nbytes = G * k * S + int(sl.sum().item())
    out["write_sources"] = {"ms": round(t, 4), "GBps": round(nbytes / t / 1e6, 1),
                            "bytes_per_launch": nbytes}
    # receive side: every source and repair packet in one slot buffer
    ps = max(sp.shape[1], rp.shape[1])
    pk = torch.zeros((G * (k + r), ps), dtype=torch.uint8, device=dev)
    pk[:G * k, :sp.shape[1]] = sp
    pk[G * k:, :rp.shape[1]] = rp
    plen = torch.cat([sl, rl])
    del sp, rp
    rb = w.read_packets(pk, plen, G, k, r, S)
    t = timed(lambda: w.read_packets(pk, plen, G, k, r, S, out=rb), a.reps, s)
    nbytes = int(plen.sum().item()) + G * (k + r) * S
    ok = bool((rb.status <= 1).all().item()) and bool((rb.src == src).all().item())
    out["read_packets"] = {"ms": round(t, 4), "GBps": round(nbytes / t / 1e6, 1),
                           "bytes_per_launch": nbytes, "verified": ok}
    for v in out.values():
        v["hbm_frac"] = round(v["GBps"] / 8000.0, 3)
    print(json.dumps({"workload": f"wire k{k}r{r}s{S} G={G}", "kernels": out}), flush=True)


if __name__ == "__main__":
    main()
