"""Per-packet C ABI (libntc.so) throughput with and without the online batching adaptor: F flows
(encoders) x M data items of S bytes, window W, rate R (a repair every R sources); the batched
run attaches every encoder to one ntc_batch_t and flushes once per round (one item per flow).
The receive side feeds each flow's packets, with 10 % i.i.d. loss, to F decoders the same way.
Prints one JSON line: packets/s of both runs on both sides (wall clock, host + PCIe + GPU).

usage: python tools/bench_batch.py [--flows 256] [--items 32] [--size 1024] [--window 32] [--rate 4]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(capi, a, batched, data):
    batch = capi.Batch() if batched else None
    encs = []
    for _ in range(a.flows):
        e = capi.Encoder()
        e.set_rate(a.rate)
        e.set_window_size(a.window)
        if batch is not None:
            e.set_batch(batch)
        encs.append(e)
    t0 = time.perf_counter()
    for i in range(a.items):
        for e in encs:
            e.add_data(data[i])
        if batch is not None:
            batch.flush()
    dt = time.perf_counter() - t0
    pk = sum(len(e.packets) for e in encs)
    rep = sum(e.nb_sent_repairs for e in encs)
    return {"s": round(dt, 4), "packets_per_s": round(pk / dt, 1), "repairs_per_s": round(rep / dt, 1),
            "packets": pk, "repairs": rep}, [e.packets for e in encs]


def run_dec(capi, batched, streams):
    batch = capi.Batch() if batched else None
    decs = []
    for _ in streams:
        d = capi.Decoder(in_order=True)
        d.set_ack_period_ms(0)
        if batch is not None:
            d.set_batch(batch)
        decs.append(d)
    rounds = max(len(s) for s in streams)
    t0 = time.perf_counter()
    for i in range(rounds):
        for d, s in zip(decs, streams):
            if i < len(s):
                d.add_packet(s[i])
        if batch is not None and i % 4 == 3:
            batch.flush()
    if batch is not None:
        batch.flush()
    dt = time.perf_counter() - t0
    npk = sum(len(s) for s in streams)
    return ({"s": round(dt, 4), "packets_per_s": round(npk / dt, 1),
             "decoded": sum(d.nb_decoded for d in decs)}, [d.data for d in decs])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flows", type=int, default=256)
    ap.add_argument("--items", type=int, default=32)
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--window", type=int, default=32)
    ap.add_argument("--rate", type=int, default=4)
    a = ap.parse_args()
    from netcode_amd import capi
    capi.load()
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, a.size, dtype=np.uint8).tobytes() for _ in range(a.items)]
    imm, p_imm = run(capi, a, False, data)
    bat, p_bat = run(capi, a, True, data)
    streams = [[p for p in flow if rng.random() >= 0.1] for flow in p_imm]
    dimm, d_imm = run_dec(capi, False, streams)
    dbat, d_bat = run_dec(capi, True, streams)
    print(json.dumps({"workload": vars(a), "encode": {"immediate": imm, "batched": bat,
                      "speedup": round(imm["s"] / bat["s"], 2), "identical_packets": p_imm == p_bat},
                      "decode": {"immediate": dimm, "batched": dbat,
                                 "speedup": round(dimm["s"] / dbat["s"], 2),
                                 "identical_deliveries": d_imm == d_bat}}), flush=True)


if __name__ == "__main__":
    main()
