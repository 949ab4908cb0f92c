"""Config 5 experiment: the dense inversion (64 dependent launches at n = 1024) eagerly vs replayed
from a captured HIP graph (torch.cuda.CUDAGraph around ntc_gf256_dense_invert_batch), and the whole
config-5 step (encode + decode) the same two ways.  One JSON line per variant.
usage: python tools/dense_graph.py [reps]
"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / reps


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from netcode_amd import DenseCode
    from netcode_amd import _native
    dev = torch.device("cuda", 0)
    G, k, S = 1, 1024, 65536
    gen = torch.Generator(device=dev).manual_seed(4321)
    src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=gen)
    dc = DenseCode(dev)
    while True:
        mat = torch.randint(0, 256, (G, k, k), dtype=torch.uint8, device=dev, generator=gen)
        _, ok = dc.invert(mat)
        if bool((ok != 0).all()):
            break
    inv = torch.empty((G, k, k), dtype=torch.uint8, device=dev)
    okb = torch.empty((G,), dtype=torch.uint8, device=dev)
    rep = torch.empty((G, k, S), dtype=torch.uint8, device=dev)
    out = torch.empty_like(src)
    L = _native.load()
    h = dc.engine.handle

    def invert():
        _native.check(L.ntc_gf256_dense_invert_batch(h, G, k, mat.data_ptr(), inv.data_ptr(), okb.data_ptr(),
                                                     torch.cuda.current_stream().cuda_stream), "invert")

    def step():
        dc.encode(mat, src, rep)
        dc.decode(mat, rep, out, okb)

    ref_inv = dc.invert(mat)[0]
    res = {"invert_eager_ms": timed(invert, reps)}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        invert()                                   # workspace allocated before capture
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            invert()
    torch.cuda.synchronize()
    inv.zero_()
    g.replay()
    torch.cuda.synchronize()
    res["invert_graph_equal"] = bool(torch.equal(inv, ref_inv))
    res["invert_graph_ms"] = timed(g.replay, reps)
    res["step_eager_ms"] = timed(step, reps)
    with torch.cuda.stream(s):
        step()
        torch.cuda.synchronize()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s):
            step()
    torch.cuda.synchronize()
    out.zero_()
    g2.replay()
    torch.cuda.synchronize()
    res["step_graph_bit_exact"] = bool(torch.equal(out, src))
    res["step_graph_ms"] = timed(g2.replay, reps)
    res["GiBps_eager"] = round(G * k * S / 2**30 / (res["step_eager_ms"] * 1e-3), 2)
    res["GiBps_graph"] = round(G * k * S / 2**30 / (res["step_graph_ms"] * 1e-3), 2)
    print(json.dumps({k_: (round(v, 4) if isinstance(v, float) else v) for k_, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
