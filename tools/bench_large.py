"""Large-window batch decode timing (decode_plan_big, 64 < r <= 255): one JSON line.

usage: python tools/bench_large.py [--k 512] [--r 255] [--m 200] [--S 1504] [--G 512]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--k", type=int, default=512)
    p.add_argument("--r", type=int, default=255)
    p.add_argument("--m", type=int, default=200)
    p.add_argument("--S", type=int, default=1504)
    p.add_argument("--G", type=int, default=512)
    p.add_argument("--reps", type=int, default=5)
    a = p.parse_args()
    from netcode_amd import BatchDecoder, BatchEncoder, status_to_numpy
    from netcode_amd import _native
    d = torch.device("cuda", 0)
    G, k, r, m, S = a.G, a.k, a.r, a.m, a.S
    gen = torch.Generator(device=d).manual_seed(7)
    src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=d, generator=gen)
    slen = torch.full((G, k), S, dtype=torch.int16, device=d)
    rng = np.random.default_rng(8)
    mask = np.ones((G, k), np.uint8)
    for g in range(G):
        mask[g, rng.choice(k, m, replace=False)] = 0
    smask = torch.from_numpy(mask).to(d)
    rmask = torch.ones((G, r), dtype=torch.uint8, device=d)
    enc, dec = BatchEncoder(k, r, d), BatchDecoder(k, r, d)
    out = enc(src, slen)
    rx = src * smask[:, :, None]
    rxl = slen * smask.to(torch.int16)
    st = torch.empty((G, 12), dtype=torch.uint8, device=d)
    L, s = _native.load(), torch.cuda.current_stream(d)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    t_plan, t_apply = [], []
    for i in range(a.reps + 1):
        x, xl = rx.clone(), rxl.clone()
        ev[0].record(s)
        _native.check(L.ntc_gf256_decode_plan(enc.engine.handle, G, k, r, xl.data_ptr(), smask.data_ptr(),
                                              out.encoded_size.data_ptr(), rmask.data_ptr(), None, None,
                                              st.data_ptr(), s.cuda_stream), "plan")
        ev[1].record(s)
        _native.check(L.ntc_gf256_decode_apply(enc.engine.handle, G, k, r, S, x.data_ptr(),
                                               out.repairs.data_ptr(), s.cuda_stream), "apply")
        ev[2].record(s)
        torch.cuda.synchronize(d)
        if i:
            t_plan.append(ev[0].elapsed_time(ev[1]))
            t_apply.append(ev[1].elapsed_time(ev[2]))
    stn = status_to_numpy(st)
    ok = torch.from_numpy(stn["state"] == 0).to(d)
    exact = bool((x[ok] == src[ok]).all())
    plan, apply_ = float(np.mean(t_plan)), float(np.mean(t_apply))
    print(json.dumps({"workload": f"k{k}r{r}m{m}s{S}", "G": G, "decoded": int(ok.sum()),
                      "bit_exact_round_trip": exact, "plan_ms": round(plan, 4),
                      "apply_ms": round(apply_, 4),
                      "decode_GiBps": round(G * k * S / ((plan + apply_) * 1e-3) / 2**30, 2),
                      "byte_mac_rate_T_per_s": round(G * m * k * S / (apply_ * 1e-3) / 1e12, 2)}))


if __name__ == "__main__":
    main()
