"""Config 5 experiment: the dense inversion (depends only on the matrix) beside the encode MAC.

Variants, each timed over N steps after a warmup (one JSON line each):
  serial      encode(mat) ; decode(mat)                      (the current bench step)
  split       encode(mat) ; invert(mat) ; encode(inv)        (same stream: the split costs nothing)
  overlap     invert(mat) on stream B  ||  encode(mat) on A ; A waits B ; encode(inv) on A
  overlapRN   the same with A created by hipExtStreamCreateWithCUMask leaving N CUs free
Checks out == src after each variant.  usage: python tools/dense_overlap.py [steps]
"""
import ctypes as C
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def masked_stream(reserve):
    hip = C.CDLL("libamdhip64.so")
    n = torch.cuda.get_device_properties(0).multi_processor_count
    words = (n + 31) // 32
    mask = (C.c_uint32 * words)()
    for cu in range(n - reserve):
        mask[cu // 32] |= 1 << (cu % 32)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), words, mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value), n


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from netcode_amd import DenseCode
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
    rep = torch.empty((G, k, S), dtype=torch.uint8, device=dev)
    out = torch.empty_like(src)
    inv = torch.empty((G, k, k), dtype=torch.uint8, device=dev)
    okb = torch.empty((G,), dtype=torch.uint8, device=dev)
    L = __import__("netcode_amd._native", fromlist=["load"]).load()
    h = dc.engine.handle

    def invert_on(stream):
        L.ntc_gf256_dense_invert_batch(h, G, k, mat.data_ptr(), inv.data_ptr(), okb.data_ptr(),
                                       stream.cuda_stream)

    def run(name, step):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        good = bool(torch.equal(out, src))
        out.zero_()
        torch.cuda.synchronize()
        gib = G * k * S / 2**30 / (ms * 1e-3)
        print(json.dumps({"variant": name, "ms_per_step": round(ms, 4), "GiBps": round(gib, 2),
                          "bit_exact": good}), flush=True)

    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def serial():
        dc.encode(mat, src, rep)
        dc.decode(mat, rep, out, okb)

    def split():
        dc.encode(mat, src, rep)
        invert_on(main_s)
        dc.encode(inv, rep, out)

    def make_overlap(A):
        def step():
            side.wait_stream(A)                   # the previous apply has read inv
            invert_on(side)
            with torch.cuda.stream(A):
                dc.encode(mat, src, rep)
                A.wait_stream(side)
                dc.encode(inv, rep, out)
        return step

    run("serial", serial)
    run("split", split)
    run("overlap", make_overlap(main_s))
    for r in (4, 8, 16, 32):
        A, n = masked_stream(r)
        run(f"overlapR{r}_of{n}", make_overlap(A))


if __name__ == "__main__":
    main()
