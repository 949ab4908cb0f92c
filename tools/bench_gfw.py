"""Throughput of the GF(2^w) batched combine (both kernel forms: the table lookups and the masked
shift-and-add, NTC_GFW_KERNEL) (ntc_gf_combine_batch, w in {4, 8, 16, 32}) at the
config-2 shape (k=32 inputs -> 8 outputs, 1 KiB symbols, G=4096), HIP events on the engine's
stream; prints one JSON line.  For comparison the GF(2^8)-dedicated batch kernels run the same
shape (ntc_gf256_combine_batch).  bytes/launch = inputs read + outputs written.

usage: python tools/bench_gfw.py [--G 4096] [--reps 10]
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
    ap.add_argument("--w", type=int, nargs="*", default=[4, 8, 16, 32])
    ap.add_argument("--forms", nargs="*", default=["fr", "mask"])
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--no-gf256", action="store_true")
    a = ap.parse_args()
    from netcode_amd import _native, combine
    from netcode_amd.engine import Engine
    dev = torch.device("cuda", 0)
    G, k, rows, S = a.G, 32, a.rows, 1024
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=g)
    s = torch.cuda.current_stream(dev)
    nbytes = G * (k + rows) * S
    out = {}
    for w in a.w:
        hi = (1 << w) - 1 if w < 32 else 2 ** 31 - 1
        cf = torch.randint(1, hi, (G, k, rows), dtype=torch.int64, device=dev, generator=g).to(torch.int32)
        res = {}
        # both kernel forms, interleaved twice: table lookups (default) and masked shift-and-add;
        # their outputs must agree
        for rep in range(2):
            for form in a.forms:
                os.environ["NTC_GFW_KERNEL"] = form
                o = combine(w, x, cf)
                t = timed(lambda: combine(w, x, cf, o), a.reps, s)
                res.setdefault(form, []).append(t)
                res.setdefault(form + "_out", o)
        os.environ.pop("NTC_GFW_KERNEL", None)
        same = bool(torch.equal(res["fr_out"], res["mask_out"])) if len(a.forms) == 2 else None
        for form in a.forms:
            t = min(res[form])
            out[f"w{w}" + ("" if form == "fr" else "_mask")] = {
                "ms": round(t, 4), "GBps": round(nbytes / t / 1e6, 1),
                "elem_MAC_T_per_s": round(G * k * rows * S * 8 / w / t / 1e9, 2),
                "all_ms": [round(v, 4) for v in res[form]]}
        if same is not None:
            out[f"w{w}"]["forms_bit_exact"] = same
    # the dedicated GF(2^8) path on the same shape
    L = _native.load()
    eng = Engine.get(dev)
    pitch = L.ntc_gf256_coef_pitch(rows)
    cf8 = torch.randint(1, 256, (G, k, pitch), dtype=torch.uint8, device=dev, generator=g)
    o8 = torch.empty((G, rows, S), dtype=torch.uint8, device=dev)
    run = lambda: _native.check(L.ntc_gf256_combine_batch(eng.handle, G, k, rows, S, x.data_ptr(),
                                                          cf8.data_ptr(), o8.data_ptr(),
                                                          s.cuda_stream), "combine")
    t = timed(run, a.reps, s)
    out["gf256_dedicated"] = {"ms": round(t, 4), "GBps": round(nbytes / t / 1e6, 1),
                              "elem_MAC_T_per_s": round(G * k * rows * S / t / 1e9, 2)}
    print(json.dumps({"workload": f"combine G={G} k={k} rows={rows} S={S}", "kernels": out}),
          flush=True)


if __name__ == "__main__":
    main()
