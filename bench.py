#!/usr/bin/env python3
"""Device-resident GF(256) encode+decode throughput (BASELINE.json metric) on MI355X.

One step = encode G generations (k sources -> r repairs) + decode the same G generations with
m lost sources each (received sources + repairs -> recovered sources), all buffers resident in
HBM.  value = G*k*S payload bytes per step / step time (GiB/s), aggregated over ranks.

Multi-GPU (torchrun): every rank owns G independent generations with its own id range (weak
scaling, no data-path collective); only a barrier and a max-reduce of the timing cross ranks, over
gloo (host tensors): no RCCL initialisation is needed for the N-GPU launch.

Extras in the JSON line:
* the timed steps run bare (no events: timing every launch costs 1.5 % of a config-3 step and
  12-15 % of a config-2 step); roofline / kernels_ms come from steps run right after them in
  which only one kernel kind at a time carries event pairs (stamped by its dispatches,
  hipExtLaunchKernelGGL, engine timing log), and kernels_fit_in_step checks their sum against
  the bare timed step (the all-stamped breakdown is reported beside them);
* roofline.traffic / valu_profile: HBM bytes and SQ instruction counts of the same kernel from
  separate rocprofv3 --pmc passes (they cannot run inside this process), labelled with the file
  and the commit they were measured at;
* an HBM copy probe of this device, the host-resident rate (pinned H2D + kernels + D2H);
* cpu_baseline: the oracle's AVX2 split-nibble path on this host, bounded sample, 1 core and all
  the cores this process may use, with the CPU model.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (k, r, S, stride, m, G)  -- BASELINE.json configs[1..3]
    "k32r8s1024": (32, 8, 1024, 1024, 8, 4096),
    "k128r32s4096": (128, 32, 4096, 4096, 32, 4096),
    "k128r32s1500": (128, 32, 1500, 1504, 32, 8192),
    # BASELINE configs[4] (extension): dense non-reference code, all k sources lost
    "k1024dense": (1024, 1024, 65536, 65536, 1024, 1),
}
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9   # CUs x SIMDs x lanes/clk x 2.4 GHz


def metric_name(config, k, r, S):
    """BASELINE.json's metric string for its headline config (config 3), the same wording with
    the workload's own shape for the others."""
    if config == "k128r32s4096":
        return "device-resident GF(256) encode+decode GiB/s, k=128 r=32, 4 KiB pkts, 1/2/4/8 GPU"
    if config == "k1024dense":
        return f"device-resident GF(256) dense encode+decode GiB/s, k={k} (all lost), {S // 1024} KiB pkts"
    size = f"{S // 1024} KiB" if S % 1024 == 0 else f"{S} B"
    return f"device-resident GF(256) encode+decode GiB/s, k={k} r={r}, {size} pkts, 1/2/4/8 GPU"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=40)
    p.add_argument("--warmup", type=int, default=30)
    p.add_argument("--config", default="k128r32s4096", choices=sorted(CONFIGS))
    p.add_argument("--G", type=int, default=0, help="generations per GPU (default per config)")
    p.add_argument("--S", type=int, default=0, help="symbol bytes (exploration; default per config)")
    p.add_argument("--stride", type=int, default=0, help="row pitch in HBM (multiple of 16, >= S; default per config)")
    p.add_argument("--r", type=int, default=0, help="repairs per generation (exploration; m capped at r)")
    p.add_argument("--mixed", action="store_true", help="m ~ U[0, r] instead of m = r")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-rate", action="store_true")
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--graph", action="store_true",
                   help="replay the step from a captured HIP graph (exploration; recorded in the line)")
    p.add_argument("--mac", default="auto", choices=("auto", "perm", "bitslice"),
                   help="region-MAC formulation (exploration; the line records it when not auto)")
    pp = p.add_argument_group("per-packet drop-in comparison (--per-packet)")
    pp.add_argument("--per-packet", action="store_true")
    pp.add_argument("--flows", type=int, default=256)
    pp.add_argument("--items", type=int, default=32)
    pp.add_argument("--size", type=int, default=1024)
    pp.add_argument("--window", type=int, default=32)
    pp.add_argument("--rate", type=int, default=4)
    pp.add_argument("--loss", type=float, default=0.1)
    pp.add_argument("--c-items", type=int, default=128, help="items per flow of the C-level legs")
    pp.add_argument("--pp-reps", type=int, default=5, help="interleaved runs of each C-level leg (best kept)")
    return p.parse_args()


def loss_mask(G, k, m, mixed, seed):
    rng = np.random.default_rng(seed)
    mask = np.ones((G, k), np.uint8)
    keys = rng.random((G, k)).argsort(axis=1)
    ms = rng.integers(0, m + 1, size=G) if mixed else np.full(G, m)
    for mm in np.unique(ms):
        rows = np.nonzero(ms == mm)[0]
        if mm:
            mask[rows[:, None], keys[rows, :mm]] = 0
    return mask


class Workload:
    def __init__(self, dev, G, k, r, S, stride, m, mixed, rank):
        from netcode_amd import BatchDecoder, BatchEncoder
        self.dev, self.G, self.k, self.r, self.S, self.stride, self.m = dev, G, k, r, S, stride, m
        gen = torch.Generator(device=dev).manual_seed(1234 + rank)
        self.src = torch.randint(0, 256, (G, k, stride), dtype=torch.uint8, device=dev, generator=gen)
        if stride != S:
            self.src[:, :, S:] = 0
        self.src_len = torch.full((G, k), S, dtype=torch.int16, device=dev)
        from netcode_amd.shard import generation_shard
        world = int(os.environ.get("WORLD_SIZE", "1"))
        sid, rid = generation_shard(rank, world, G, k, r)
        self.sid = torch.from_numpy(sid.view(np.int32)).to(dev)
        self.rid = torch.from_numpy(rid.view(np.int32)).to(dev)
        mask = loss_mask(G, k, m, mixed, 99 + rank)
        self.nlost = int((mask == 0).sum())
        self.smask = torch.from_numpy(mask).to(dev)
        self.rmask = torch.ones((G, r), dtype=torch.uint8, device=dev)
        self.rx = self.src * self.smask[:, :, None]            # decoder-side slots
        self.rx_len = self.src_len * self.smask.to(torch.int16)
        self.enc = BatchEncoder(k, r, dev)
        self.dec = BatchDecoder(k, r, dev)
        self.out = None
        self.status = torch.empty((G, 12), dtype=torch.uint8, device=dev)
        self.enc.engine.reserve(G, k, r)

    def step(self):
        self.out = self.enc(self.src, self.src_len, self.sid, self.rid, self.out)
        self.dec(self.rx, self.rx_len, self.smask, self.out.repairs, self.out.encoded_size,
                 self.rmask, self.sid, self.rid, self.status)

    POISON = 0xA5

    def poison(self):
        """Before the last profiled step: every output of the step is overwritten with a poison
        byte -- the lost source slots (the decoder's in-place outputs), the repairs, the encoded
        sizes, the status words -- after keeping the previous step's repairs / sizes / status.
        Steps are deterministic, so after the step `rewritten()` proves the step recomputed all
        of them (a skipped or partial launch would leave poison behind)."""
        self._prev = (self.out.repairs.clone(), self.out.encoded_size.clone(), self.status.clone())
        self.rx[self.smask == 0] = self.POISON
        self.out.repairs.fill_(self.POISON)
        self.out.encoded_size.fill_(-23131)            # 0xA5A5
        self.status.fill_(self.POISON)

    def rewritten(self):
        rep, esz, st = self._prev
        from netcode_amd import status_to_numpy
        dec = torch.from_numpy(status_to_numpy(self.status)["state"] == 0).to(self.dev)
        lost = (self.smask == 0) & dec[:, None]
        ok = (torch.equal(self.out.repairs, rep) and torch.equal(self.out.encoded_size, esz) and
              torch.equal(self.status, st) and bool((self.rx[lost] == self.src[lost]).all()))
        self._prev = None
        return ok

    def oracle_sample(self, n=24, n_singular=8):
        """Host copies of a sample of generations of the last step (evenly spaced + the first
        singular ones), for the oracle comparison of the cpu_baseline leg."""
        from netcode_amd import status_to_numpy
        st = status_to_numpy(self.status)
        g = set(np.linspace(0, self.G - 1, min(n, self.G)).astype(int).tolist())
        g |= set(np.nonzero(st["state"] == 3)[0][:n_singular].tolist())
        g = np.array(sorted(g))
        gi = torch.from_numpy(g).to(self.dev)
        h = lambda t: t.index_select(0, gi).cpu().numpy()
        return {"g": g, "src": h(self.src), "len": h(self.src_len).view(np.uint16),
                "mask": h(self.smask), "rmask": h(self.rmask), "sid": h(self.sid).view(np.uint32),
                "rid": h(self.rid).view(np.uint32), "rep": h(self.out.repairs),
                "esz": h(self.out.encoded_size).view(np.uint16), "rx": h(self.rx),
                "rx_len": h(self.rx_len).view(np.uint16), "status": st[g], "k": self.k, "r": self.r}

    def verify(self):
        """(bit-exact, decoded generations, decode MAC bytes, decode byte-MACs) of the last step.
        Every generation with a loss must end decoded or singular (all repairs arrive and m <= r,
        so "not enough repairs" is impossible) with at most 10 % singular (the reference schedule
        gives ~2 % at k=128/m=32), every loss-free one "nothing missing", and every decoded one
        must equal its sources bit for bit."""
        from netcode_amd import status_to_numpy
        st = status_to_numpy(self.status)
        dec = st["state"] == 0
        ok = torch.from_numpy(dec).to(self.dev)
        good = bool((self.rx[ok] == self.src[ok]).all())
        lossy = st["nb_missing"] > 0            # m = 0 (mixed runs): "nothing missing" is right
        allowed = np.where(lossy, np.isin(st["state"], (0, 3)), st["state"] == 1)
        good = bool(good and allowed.all() and dec[lossy].mean() >= 0.9)
        m = st["nb_missing"].astype(np.int64)[dec]
        # decode MAC per decoded generation: reads (k - m) received sources + m repairs, writes m
        dec_bytes = int(((self.k + m) * self.S).sum())
        dec_macs = int((m * self.k * self.S).sum())
        return good, int(dec.sum()), dec_bytes, dec_macs


class DenseWorkload:
    """BASELINE config 5: k = 1024 sources of 64 KiB, all lost; 1024 repairs from a seeded dense
    random GF(2^8) matrix (re-drawn if singular).  Step = dense encode + dense decode (device
    Gauss-Jordan of the 1024 x 1024 matrix + the MAC with its inverse)."""

    def __init__(self, dev, G, k, S, rank):
        from netcode_amd import DenseCode
        self.dev, self.G, self.k, self.r, self.S, self.stride, self.m = dev, G, k, k, S, S, k
        self.nlost = G * k
        gen = torch.Generator(device=dev).manual_seed(4321 + rank)
        self.src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=dev, generator=gen)
        self.dc = DenseCode(dev)
        while True:
            self.mat = torch.randint(0, 256, (G, k, k), dtype=torch.uint8, device=dev, generator=gen)
            _, ok = self.dc.invert(self.mat)
            if bool((ok != 0).all()):
                break
        self.rep = torch.empty((G, k, S), dtype=torch.uint8, device=dev)
        self.out = torch.empty_like(self.src)
        self.ok = torch.empty((G,), dtype=torch.uint8, device=dev)

    def poison(self):
        """Before the last profiled step: the decoded-source buffer and the repairs are poisoned
        (after keeping the previous step's repairs); see Workload.poison."""
        self._prev = self.rep.clone()
        self.out.fill_(0xA5)
        self.rep.fill_(0xA5)
        self.ok.fill_(0)

    def rewritten(self):
        ok = torch.equal(self.rep, self._prev) and torch.equal(self.out, self.src)
        self._prev = None
        return ok

    def oracle_sample(self):
        return None

    def step(self):
        self.dc.encode(self.mat, self.src, self.rep)
        self.dc.decode(self.mat, self.rep, self.out, self.ok)

    def verify(self):
        good = bool((self.ok != 0).all().item()) and bool(torch.equal(self.out, self.src))
        n = int((self.ok != 0).sum().item())
        # the decode MAC reads the k repairs and writes the k sources of each generation
        return good, n, n * 2 * self.k * self.S, n * self.k * self.k * self.S


def hbm_copy_probe(dev, nbytes=1 << 30, reps=5):
    """Device-to-device copy bandwidth (read + write bytes / time), GB/s: confirms the HBM peak
    the roofline divides by on this very device."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    s = torch.cuda.current_stream(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(s)
    for _ in range(reps):
        b.copy_(a)
    ev[1].record(s)
    torch.cuda.synchronize(dev)
    ms = ev[0].elapsed_time(ev[1]) / reps
    del a, b
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


def host_rate(w, reps=3):
    """Host-resident rate (PCIe-inclusive GiB/s of source payload), never `value`: sources start
    in pinned host memory, repairs and recovered sources end there.  Returns (packed, pipelined,
    serial, packed_ok): packed = HostPipeline.encode_decode_packed (only the received sources go
    H2D for the decoder and only the lost slots come back, packed -- what a real receiver moves);
    pipelined = HostPipeline.encode_decode over whole generation slots (chunks of G/16
    generations over 3 HIP streams, so H2D, kernels and D2H of different chunks overlap); serial =
    one H2D -> encode -> D2H -> H2D -> decode -> D2H pass over the whole batch; packed_ok = the
    packed run's recovered rows equal the lost sources of every decoded generation."""
    from netcode_amd.pipeline import HostPipeline
    dev = w.dev
    pin = lambda t: torch.empty_like(t, device="cpu").pin_memory().copy_(t)
    h_src, h_len, h_rx, h_rxlen = pin(w.src), pin(w.src_len), pin(w.rx), pin(w.rx_len)
    h_mask, h_rmask = pin(w.smask), pin(w.rmask)
    h_rep = torch.empty((w.G, w.r, w.stride), dtype=torch.uint8).pin_memory()
    h_rsz = torch.empty((w.G, w.r), dtype=torch.int16).pin_memory()
    h_st = torch.empty((w.G, 12), dtype=torch.uint8).pin_memory()
    d_src = torch.empty_like(w.src)
    d_rx = torch.empty_like(w.rx)
    torch.cuda.synchronize(dev)

    def best(fn):
        times = []
        for _ in range(reps + 1):              # first pass warms the streams / engines
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t0)
        return w.G * w.k * w.S / min(times[1:]) / 2**30

    def serial():
        d_src.copy_(h_src, non_blocking=True)
        out = w.enc(d_src, w.src_len, w.sid, w.rid, w.out)
        h_rep.copy_(out.repairs, non_blocking=True)
        d_rx.copy_(h_rx, non_blocking=True)
        w.dec(d_rx, w.rx_len, w.smask, out.repairs, out.encoded_size, w.rmask, w.sid, w.rid,
              w.status)
        h_rx.copy_(d_rx, non_blocking=True)

    pipe = HostPipeline(w.k, w.r, w.stride, max(1, w.G // 16), dev, depth=3)

    def pipelined():
        pipe.encode_decode(h_src, h_len, h_rep, h_rsz, h_rx, h_rxlen, h_mask, h_rmask, h_st,
                           w.sid, w.rid)

    mask_h = w.smask.cpu()
    _, _, n_rx, n_lost = HostPipeline.row_bases(mask_h)
    keep = mask_h.bool()
    h_rxp = w.src.cpu()[keep].contiguous().pin_memory()
    h_rec = torch.empty((n_lost, w.stride), dtype=torch.uint8).pin_memory()

    def packed():
        pipe.encode_decode_packed(h_src, h_len, h_rep, h_rsz, h_rxp, h_rxlen, h_mask, h_rmask,
                                  h_rec, h_st, w.sid, w.rid)

    rate_serial = best(serial)
    rate_pipe = best(pipelined)
    h_rxlen.copy_(w.rx_len.cpu())
    rate_packed = best(packed)
    from netcode_amd import status_to_numpy
    dec = torch.from_numpy(status_to_numpy(h_st)["state"] == 0)
    lost_gen = torch.nonzero(~keep)[:, 0]          # generation of every packed lost row
    want = w.src.cpu()[~keep]
    sel = dec[lost_gen]
    packed_ok = bool(sel.any()) and bool((h_rec[sel] == want[sel]).all())
    return rate_packed, rate_pipe, rate_serial, packed_ok


# The bit-sliced chain alone (the product's shared-table chain, no fill, no memory stream) on
# MI355X: 51.5 cycles per 2048-byte-MAC wave-row per SIMD = 98 T byte-MAC/s
# (profiles/r03/microbench_chain_README.md, tools/gen_microbench_chain.py).
CHAIN_PEAK_TBMAC = 98.0
CHAIN_PEAK_SOURCE = ("chain microbenchmark, product chain R8 W4: 51.5 cycles/row/SIMD = 98 T "
                     "byte-MAC/s (profiles/r03/microbench_chain_README.md)")


def cpu_info():
    """(model name, nproc of this machine, CPUs this process may run on)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return model, os.cpu_count() or 1, usable


def cpu_quota():
    """The cgroup CPU bandwidth limit of this process in CPUs (cgroup v2 cpu.max, v1 cfs quota),
    or None when unlimited / unreadable: the affinity mask can list every CPU of the machine while
    the scheduler grants only a share of them."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            txt = open(path).read().strip()
        except OSError:
            continue
        if parse:
            q, per = parse(txt)
            return None if q == "max" else round(int(q) / int(per), 2)
        q = int(txt)
        if q <= 0:
            return None
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return round(q / per, 2)
    return None


def effective_cpus():
    """CPUs this process can actually use: the affinity mask, capped by the cgroup CPU quota
    (a gpurun box lists every CPU of the machine in the mask but grants 16 of them)."""
    _, _, usable = cpu_info()
    q = cpu_quota()
    return max(1, min(usable, int(q))) if q else usable


def cpu_baseline_run(k, r, S, stride, m, threads, budget_s):
    """One timed CPU leg: encode + decode of a bounded sample of the workload shape with the
    oracle's AVX2 split-nibble region MAC (encode: the repair loop of detail/encoder.cc:15-64;
    decode: the reference's streaming decoder state machine, detail/decoder.cc, fed the received
    sources then the repairs).  Returns (GiB/s of payload, sample description, t_enc, t_dec)."""
    from oracle import oracle as O
    G = 8
    rng = np.random.default_rng(7)
    src = rng.integers(0, 256, (G, k, stride), dtype=np.uint8)
    src[:, :, S:] = 0
    lens = np.full((G, k), S, np.uint16)
    mask = loss_mask(G, k, m, False, 8)
    rmask = np.ones((G, r), np.uint8)
    # calibrate on one generation (single thread), then size the sample to the budget
    t0 = time.perf_counter()
    rep, rsz = O.encode_batch(src[:1], lens[:1], k, r, simd=True, threads=1)
    lost = src[:1] * mask[:1, :, None]
    O.decode_batch(lost, lens[:1] * mask[:1], mask[:1], rep, rsz, rmask[:1])
    per_gen = time.perf_counter() - t0
    Gs = int(max(threads, min(1024, budget_s / max(per_gen, 1e-6) * threads / 4)))
    Gs = max(threads, (Gs // threads) * threads)
    src = np.ascontiguousarray(np.broadcast_to(src[:1], (Gs, k, stride)))
    lens = np.full((Gs, k), S, np.uint16)
    mask = loss_mask(Gs, k, m, False, 9)
    rmask = np.ones((Gs, r), np.uint8)
    lost = src * mask[:, :, None]
    llen = lens * mask
    t_enc = t_dec = 0.0
    passes = 0
    while passes < 1 or (t_enc + t_dec < budget_s and passes < 64):
        t0 = time.perf_counter()
        rep, rsz = O.encode_batch(src, lens, k, r, simd=True, threads=threads)
        t1 = time.perf_counter()
        O.decode_batch(lost, llen, mask, rep, rsz, rmask, threads=threads)
        t2 = time.perf_counter()
        t_enc += t1 - t0
        t_dec += t2 - t1
        passes += 1
    gib = passes * Gs * k * S / 2**30
    return gib / (t_enc + t_dec), f"{passes} x {Gs} generations", t_enc, t_dec


def cpu_baseline(k, r, S, stride, m, threads, budget_s=12.0):
    """Oracle's AVX2 split-nibble path (gf-complete's w=8 algorithm class; gf-complete itself is
    not in the image), same workload shape, bounded samples on 1 core and on `threads` cores;
    returns the dict for the JSON line (value = the all-core leg)."""
    from oracle import oracle as O
    L = O.lib()
    L.or_set_simd(1)
    model, nproc, usable = cpu_info()
    try:
        v1, s1, e1, d1 = cpu_baseline_run(k, r, S, stride, m, 1, budget_s / 3)
        vn, sn, en, dn = cpu_baseline_run(k, r, S, stride, m, threads, budget_s * 2 / 3)
        gfni = None
        if L.or_have_gfni():
            # labelled upper bound: GFNI affine-matrix region MACs, AVX-512
            L.or_set_simd(2)
            g1 = cpu_baseline_run(k, r, S, stride, m, 1, budget_s / 6)
            gn = cpu_baseline_run(k, r, S, stride, m, threads, budget_s / 3)
            gfni = {"value": round(gn[0], 3), "unit": "GiB/s", "cores": threads,
                    "sample": gn[1], "encode_s": round(gn[2], 3), "decode_s": round(gn[3], 3),
                    "single_core": {"value": round(g1[0], 3), "sample": g1[1]},
                    "note": "upper-bound leg, not gf-complete's algorithm: the same oracle with "
                            "each region MAC as gf2p8affineqb over 64-byte vectors"}
    finally:
        L.or_set_simd(0)
    shape = f"k={k} r={r} S={S} m={m}, encode+decode"
    return {"value": round(vn, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{sn} {shape} on {threads} threads ({en + dn:.1f}s wall); AVX2 split-nibble "
                      f"oracle path (gf-complete w=8 algorithm class); decode = the reference's "
                      f"streaming decoder state machine (per-packet buffers, repair reduction, "
                      f"inversion), hence slower than encode at equal MAC counts",
            "encode_s": round(en, 3), "decode_s": round(dn, 3),
            "single_core": {"value": round(v1, 3), "cores": 1, "sample": f"{s1} {shape}",
                            "encode_s": round(e1, 3), "decode_s": round(d1, 3)},
            "gfni_upper_bound": gfni,
            "cpu_model": model, "nproc": nproc, "usable_cpus": usable,
            "cgroup_cpu_quota": cpu_quota(), "effective_cpus": effective_cpus(),
            "cores_note": "cores = the threads of the all-core leg = the effective CPU count "
                          "(affinity mask capped by the cgroup quota)"}


def _pp_encode(mk_enc, a, data, batch=None):
    """Per-packet encode leg: F flows x M items through the reference's encoder API (one
    add_data per item and flow, round-robin over flows; a batch is flushed once per round)."""
    encs = []
    for _ in range(a.flows):
        e = mk_enc()
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
    return {"s": round(dt, 4), "packets_per_s": round(pk / dt, 1), "packets": pk,
            "repairs": sum(e.nb_sent_repairs for e in encs)}, [list(e.packets) for e in encs]


def _pp_decode(mk_dec, streams, batch=None):
    """Per-packet decode leg: every flow's surviving packets fed to its own in-order decoder,
    round-robin over flows (batch flushed every 4 rounds and at the end)."""
    decs = []
    for _ in streams:
        d = mk_dec()
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
    got = [[x[1] if isinstance(x, tuple) else x for x in d.data] for d in decs]
    return {"s": round(dt, 4), "packets_per_s": round(npk / dt, 1),
            "decoded": sum(d.nb_decoded for d in decs)}, got


def per_packet_main(a):
    """Drop-in comparison at the reference's own API granularity (verdict r1 #7): the C ABI
    (libntc.so, include/netcode/c/*.h; the GPU combine behind ntc_encoder_add_data /
    ntc_decoder_add_packet, immediate and through ntc_batch_t) against the oracle's restatement
    of ntc::encoder / ntc::decoder with its AVX2 region ops, on the same per-flow streams (the
    reference's usage: one object per flow, one call per packet; the Python driver loop is
    identical for both).  Prints one JSON line; `value` = batched GPU encode+decode packets/s
    (eager batches, synchronous flushes); the asynchronous-flush leg is reported beside it."""
    from netcode_amd import capi
    from oracle import oracle as O
    import __graft_entry__
    __graft_entry__.build()
    capi.load()
    rng = np.random.default_rng(0)
    data = [rng.integers(0, 256, a.size, dtype=np.uint8).tobytes() for _ in range(a.items)]
    imm, p_imm = _pp_encode(capi.Encoder, a, data)
    bat, p_bat = _pp_encode(capi.Encoder, a, data, capi.Batch())
    L = O.lib()
    L.or_set_simd(1)
    try:
        cpu, p_cpu = _pp_encode(O.Encoder, a, data)
        streams = [[p for p in flow if rng.random() >= a.loss] for flow in p_imm]
        dcpu, d_cpu = _pp_decode(lambda: O.Decoder(in_order=True), streams)
    finally:
        L.or_set_simd(0)
    dimm, d_imm = _pp_decode(lambda: capi.Decoder(in_order=True), streams)
    dbat, d_bat = _pp_decode(lambda: capi.Decoder(in_order=True), streams, capi.Batch())
    n_enc, n_dec = imm["packets"], sum(len(s) for s in streams)
    both = lambda e, d: round((n_enc + n_dec) / (e["s"] + d["s"]), 1)
    py_ok = p_cpu == p_imm == p_bat and d_cpu == d_imm == d_bat

    # C level: the same loop in C on both sides (tools/pp_driver.c over libntc.so; the oracle's
    # or_pp_bench), same payload / loss draws, packets and deliveries compared by hash
    import subprocess
    drv = os.path.join(ROOT, "tests", "_build", "pp_driver")
    cargs = [str(x) for x in (a.flows, a.c_items, a.size, a.window, a.rate, int(round(a.loss * 100)), 7)]
    # each C-level leg runs `reps` times, interleaved (host load on the box drifts), best kept
    def run_gpu(mode):
        out = subprocess.run([drv, mode] + cargs, capture_output=True, text=True, timeout=600)
        if out.returncode != 0:
            raise RuntimeError(f"pp_driver {mode} failed: {out.stderr[-400:]}")
        return json.loads(out.stdout.strip().splitlines()[-1])

    def run_cpu():
        secs = (C.c_double * 2)()
        cnt = (C.c_uint64 * 4)()
        hs = (C.c_uint64 * 2)()
        L.or_set_simd(1)
        try:
            L.or_pp_bench(a.flows, a.c_items, a.size, a.window, a.rate, int(round(a.loss * 100)),
                          C.c_uint64(7), secs, cnt, hs)
        finally:
            L.or_set_simd(0)
        return {"encode_s": secs[0], "decode_s": secs[1], "packets": cnt[0], "received": cnt[1],
                "deliveries": cnt[2], "repairs": cnt[3], "packets_hash": f"{hs[0]:016x}",
                "deliveries_hash": f"{hs[1]:016x}"}

    runs = {"immediate": [], "batched": [], "async": [], "cpu": []}
    for _ in range(a.pp_reps):
        runs["batched"].append(run_gpu("batched"))
        runs["async"].append(run_gpu("async"))
        runs["cpu"].append(run_cpu())
        runs["immediate"].append(run_gpu("immediate"))
    best = lambda rs: min(rs, key=lambda r: r["encode_s"] + r["decode_s"])
    c_gpu = {m: best(runs[m]) for m in ("immediate", "batched", "async")}
    c_cpu = best(runs["cpu"])
    for m, rs in runs.items():
        (c_cpu if m == "cpu" else c_gpu[m])["all_runs_s"] = [round(r["encode_s"] + r["decode_s"], 5) for r in rs]
    cpps = lambda r: round((r["packets"] + r["received"]) / (r["encode_s"] + r["decode_s"]), 1)
    for r in list(c_gpu.values()) + [c_cpu]:
        r["packets_per_s"] = cpps(r)
    c_ok = all(r["packets_hash"] == c_cpu["packets_hash"] and
               r["deliveries_hash"] == c_cpu["deliveries_hash"] for rs in runs.values() for r in rs)
    model, _, _ = cpu_info()
    line = {"metric": "per-packet drop-in encode+decode packets/s (C ABI, one object per flow)",
            "value": c_gpu["batched"]["packets_per_s"], "unit": "packets/s", "n_gpus": 1,
            "higher_is_better": True, "vs_baseline": None, "dtype": "u8 (GF(2^8))",
            "data": f"synthetic ({a.flows} flows x {a.c_items} items of {a.size} B, window "
                    f"{a.window}, a repair every {a.rate} sources, {a.loss:.0%} i.i.d. loss)",
            "config": {"workload": "per-packet", **{k_: getattr(a, k_) for k_ in
                       ("flows", "c_items", "size", "window", "rate", "loss")}},
            "value_note": "C-level driver (tools/pp_driver.c), GPU region ops batched across flows "
                          "(ntc_batch_t, eager batches, synchronous flushes; gpu_async = the same "
                          "with asynchronous flushes, ntc_batch_set_async); packets "
                          "encoded + packets received, over encode + "
                          "decode time; best of the interleaved runs of each leg (all_runs_s); "
                          "both legs copy each item in inside the loop and write into "
                          "application stores sized and paged in before the clock",
            "c_level": {"gpu_async": c_gpu["async"], "gpu_batched": c_gpu["batched"],
                        "gpu_immediate": c_gpu["immediate"],
                        "cpu_oracle": c_cpu},
            "cpu_baseline": {"value": c_cpu["packets_per_s"], "unit": "packets/s", "cores": 1,
                             "kind": "port", "cpu_model": model,
                             "sample": "the same C-level workload through the oracle's ntc::encoder "
                                       "/ ntc::decoder restatement (AVX2 split-nibble regions)"},
            "speedup_async_vs_cpu": round(c_gpu["async"]["packets_per_s"] / c_cpu["packets_per_s"], 2),
            "speedup_batched_vs_cpu": round(c_gpu["batched"]["packets_per_s"] / c_cpu["packets_per_s"], 2),
            "speedup_immediate_vs_cpu": round(c_gpu["immediate"]["packets_per_s"] / c_cpu["packets_per_s"], 2),
            "python_level": {"items": a.items,
                             "gpu_immediate": {"encode": imm, "decode": dimm, "packets_per_s": both(imm, dimm)},
                             "gpu_batched": {"encode": bat, "decode": dbat, "packets_per_s": both(bat, dbat)},
                             "cpu_oracle": {"encode": cpu, "decode": dcpu, "packets_per_s": both(cpu, dcpu)}},
            "verified": {"c_level_packets_and_deliveries_identical": c_ok,
                         "python_level_packets_and_deliveries_identical": py_ok}}
    print(json.dumps(line), flush=True)
    if not (py_ok and c_ok):
        sys.exit(3)


def host_rate_wire(w, reps=3):
    """Host-resident rate through the WIRE format (PCIe-inclusive GiB/s of source payload, never
    `value`), socket buffer to socket buffer: sender = sources H2D -> encode -> write_repairs ->
    repair packets D2H; receiver = its received source packets + the repair packets H2D ->
    read_packets (+ _append) -> decode -> pack_slots of the lost rows -> D2H
    (HostPipeline.encode_decode_wire, chunks of G/16 over 3 streams).  Returns (GiB/s, ok, repair
    packets of the run [G*r, rps] host, lengths): ok = the repair packets equal the device-resident
    Wire.write_repairs of the same repairs, and every decoded generation's recovered rows and sizes
    equal its lost sources."""
    from netcode_amd.engine import Wire
    from netcode_amd.pipeline import HostPipeline
    dev, G, k, r, stride = w.dev, w.G, w.k, w.r, w.stride
    wire = Wire(dev)
    pin = lambda t: torch.empty_like(t, device="cpu").pin_memory().copy_(t)
    # the receiver's socket buffers: the source packets that were not lost, generation-major
    spk, slen = wire.write_sources(w.src, w.src_len, w.sid)
    keep = (w.smask.reshape(-1) != 0).nonzero().reshape(-1)
    h_rxp, h_rxl = pin(spk.index_select(0, keep)), pin(slen.index_select(0, keep))
    cnt = (w.smask != 0).sum(1).cpu().to(torch.int64)
    rx_first = torch.zeros(G + 1, dtype=torch.int64)
    rx_first[1:] = torch.cumsum(cnt, 0)
    rpk_dev, rlen_dev = wire.write_repairs(w.out, k, w.sid, w.rid)
    rps = rpk_dev.shape[1]
    h_src, h_len, h_mask = pin(w.src), pin(w.src_len), pin(w.smask)
    h_rep_pkts = torch.empty((G * r, rps), dtype=torch.uint8).pin_memory()
    h_rep_len = torch.empty((G * r,), dtype=torch.int32).pin_memory()
    _, _, _, n_lost = HostPipeline.row_bases(h_mask)
    h_rec = torch.empty((n_lost, stride), dtype=torch.uint8).pin_memory()
    h_dec_len = torch.empty((G, k), dtype=torch.int16).pin_memory()
    h_st = torch.empty((G, 12), dtype=torch.uint8).pin_memory()
    sid_h = w.sid.cpu().numpy().view(np.uint32)
    rid_h = w.rid.cpu().numpy().view(np.uint32)
    pipe = HostPipeline(k, r, stride, max(1, G // 16), dev, depth=3)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(reps + 1):                  # the first pass warms the streams / engines
        t0 = time.perf_counter()
        pipe.encode_decode_wire(h_src, h_len, h_rep_pkts, h_rep_len, h_rxp, h_rxl, rx_first, h_mask,
                                h_rec, h_dec_len, h_st, sid_h, rid_h, w.sid, w.rid)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    rate = G * k * w.S / min(times[1:]) / 2**30
    # each packet's bytes up to its length (the slot bytes past it are not part of the packet)
    d_pk, d_len = rpk_dev.cpu(), rlen_dev.cpu()
    inpkt = torch.arange(rps)[None, :] < d_len.to(torch.int64)[:, None]
    checks = {"packet_lengths": torch.equal(h_rep_len, d_len),
              "packet_bytes": torch.equal(h_rep_pkts[inpkt], d_pk[inpkt])}
    from netcode_amd import status_to_numpy
    st = status_to_numpy(h_st)
    lost = (w.smask == 0).cpu()
    dec = torch.from_numpy(st["state"] == 0)
    rec_gen = torch.repeat_interleave(torch.arange(G), lost.sum(1))   # generation of each lost row
    src_lost = w.src.cpu()[lost]
    sel = dec[rec_gen]
    checks["recovered_rows"] = torch.equal(h_rec[sel], src_lost[sel])
    checks["recovered_lengths"] = torch.equal(h_dec_len[lost][sel], w.src_len.cpu()[lost][sel])
    host_rate_wire.checks = checks
    return rate, all(checks.values()), h_rep_pkts, h_rep_len


def oracle_check(smp, threads):
    """cpu_baseline leg (the oracle is the checker here, never the measured path): the sampled
    generations of the bench's own last step against the oracle on the same sources, lengths, id
    bases and loss masks -- repairs, encoded sizes, per-generation decode status, recovered slots
    and lengths, bit for bit."""
    from oracle import oracle as O
    k, r = smp["k"], smp["r"]
    orep, orsz = O.encode_batch(smp["src"], smp["len"], k, r, smp["sid"], smp["rid"], simd=True,
                                threads=threads)
    lost = smp["src"] * smp["mask"][:, :, None]
    out, olen, ost = O.decode_batch(lost, smp["len"] * smp["mask"], smp["mask"], orep, orsz,
                                    smp["rmask"], smp["sid"], smp["rid"], threads=threads)
    # the wire leg's repair packets of these generations against the oracle's packetizer
    # (packetizer.hh:90-122) over the oracle's own repairs
    pk_ok = None
    if smp.get("rep_pkts") is not None:
        pk_ok = True
        for gi in range(len(smp["g"])):
            ids = (smp["sid"][gi].astype(np.uint64) + np.arange(k, dtype=np.uint64)) & 0xFFFFFFFF
            L = int(smp["len"][gi].max())
            for j in range(r):
                ref = O.write_repair_packet(int(smp["rid"][gi]) + j, orep[gi, j, :L], ids, int(orsz[gi, j]))
                got = smp["rep_pkts"][gi, j, :int(smp["rep_pkt_len"][gi, j])].tobytes()
                pk_ok = pk_ok and ref == got
    # slots the decoder owns: every slot of a decoded generation, the received ones otherwise (the
    # lost slots of a generation that does not decode are not written by either side)
    own = (ost["state"] == 0)[:, None] | (smp["mask"] != 0)
    res = {"repairs": bool((orep == smp["rep"]).all()), "encoded_sizes": bool((orsz == smp["esz"]).all()),
           "status": bool((ost == smp["status"]).all()),
           "decoded_slots": bool((out[own] == smp["rx"][own]).all()),
           "decoded_lengths": bool((olen == smp["rx_len"]).all()),
           **({"wire_repair_packets": pk_ok} if pk_ok is not None else {}),
           "decoded_generations": int((ost["state"] == 0).sum()),
           "singular_generations": int((ost["state"] == 3).sum())}
    return all(v for k_, v in res.items() if isinstance(v, bool)), res


def cpu_baseline_dense(w, sample_bytes=1024):
    """Config 5 CPU leg: the oracle's dense encode (region MACs, AVX2 split-nibble) and dense
    decode (the reference's jerasure-order Gauss-Jordan, invert_matrix.cc:9-128, then the MACs
    with the inverse) on the bench's own matrix, single core.  The MACs run over a `sample_bytes`
    column slice of the 64 KiB sources and scale linearly in S (the per-byte work of every MAC is
    the same); the inversion runs once, in full.  value = k*S / (t_enc_mac(S) + t_invert +
    t_dec_mac(S))."""
    from oracle import oracle as O
    L = O.lib()
    L.or_set_simd(1)
    try:
        mat = w.mat[0].cpu().numpy()
        src = np.ascontiguousarray(w.src[0, :, :sample_bytes].cpu().numpy())
        t0 = time.perf_counter()
        rep = O.dense_encode(mat, src)
        t1 = time.perf_counter()
        ok, out, inv = O.dense_decode(mat, rep)
        t2 = time.perf_counter()
        again = O.dense_encode(inv, rep)          # the decode's MAC alone (same matrix, same rows)
        t3 = time.perf_counter()
    finally:
        L.or_set_simd(0)
    t_enc, t_dmac = t1 - t0, t3 - t2
    t_inv = max(t2 - t1 - t_dmac, 0.0)
    fail = None if (again == src).all() else "mismatch"
    scale = w.S / sample_bytes
    total = t_enc * scale + t_inv + t_dmac * scale
    model, nproc, usable = cpu_info()
    return {"value": round(w.k * w.S / total / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"k={w.k} dense: encode + decode MACs over a {sample_bytes}-byte column "
                      f"slice scaled x{scale:g} to S={w.S}, plus one full {w.k}x{w.k} inversion "
                      f"(oracle, jerasure order); {t3 - t0:.1f}s wall",
            "encode_mac_s_at_S": round(t_enc * scale, 3), "invert_s": round(t_inv, 3),
            "decode_mac_s_at_S": round(t_dmac * scale, 3),
            "sample_bit_exact": bool(ok and fail is None and (out == src).all()),
            "cpu_model": model, "nproc": nproc, "usable_cpus": usable}


def kernel_summary(log, steps, dense):
    """Per-step kernel times from the timing log of the timed steps: {name: ms per step} and the
    per-launch durations of the encode / decode MAC kernels."""
    if not log or len(log) % steps:
        raise RuntimeError(f"timing log has {len(log)} entries for {steps} steps")
    per = len(log) // steps
    tot, launches = {}, {"encode_mac": [], "decode_mac": []}
    for s0 in range(0, len(log), per):
        seen_mac = seen_dense = 0
        for name, ms in log[s0:s0 + per]:
            if dense and name == "encode_mac":       # dense step: encode combine, decode combine
                name = "decode_mac" if seen_mac else "encode_mac"
                seen_mac += 1
            elif dense and name == "dense":
                name = "dense_invert" if seen_dense else "dense_encode_layout"
                seen_dense += 1
            elif name == "other":                     # the split-k MAC's part reduction
                name = "ksplit_reduce"
            elif name == "preslice":                  # a tall MAC's source pre-slicing pass
                name = "source_preslice"
            tot[name] = tot.get(name, 0.0) + ms
            if name in launches:
                launches[name].append(ms)
    return {n: v / steps for n, v in tot.items()}, launches


def pmc_record(fname, config, kernel):
    """A rocprofv3 PMC result for (config, kernel) from a committed profiles/ file, with where it
    came from (file + the commit it was measured at): these counters need their own profiler
    passes and cannot be collected inside this run."""
    path = os.path.join(ROOT, "profiles", fname)
    if not os.path.exists(path):
        return None, None
    try:
        j = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    rec = j.get(config, {}).get(kernel)
    if rec is None:
        return None, None
    ent = j.get(config, {})
    src = {"file": "profiles/" + fname,
           "commit": ent.get("_commit", j.get("_commit", "unrecorded")),
           "how": ent.get("_how", j.get("_how", "rocprofv3 --pmc passes"))}
    return rec, src


def main():
    a = parse()
    if a.per_packet:
        return per_packet_main(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU.  The ranks exchange no data: the barrier and the step-time
    # max run over gloo on host tensors, so the N-GPU launch never initialises RCCL
    # (NTC_BENCH_BACKEND=nccl selects it).  With fewer GPUs than ranks (a test), ranks share
    # devices round-robin.
    backend = os.environ.get("NTC_BENCH_BACKEND", "gloo")
    ndev = torch.cuda.device_count()
    local = local % ndev if (backend == "gloo" and ndev) else local
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # physical devices in use: ranks of a gloo test share devices round-robin
    n_gpus = min(world, ndev) if (backend == "gloo" and ndev) else world
    k, r, S, stride, m, Gdef = CONFIGS[a.config]
    if a.S:
        S, stride = a.S, (a.S + 15) // 16 * 16
    if a.stride:
        assert a.stride >= S and a.stride % 16 == 0, "--stride: a multiple of 16, at least S"
        stride = a.stride
    G = a.G or Gdef
    if a.r:                              # exploration: fewer / more repairs (m capped at r)
        r, m = a.r, min(m, a.r)

    if world == 1:
        import __graft_entry__
        __graft_entry__.build()          # no-op when the in-tree libraries are up to date
    else:
        # ranks never build concurrently: the in-tree .so files are prebuilt (build())
        import netcode_amd
        netcode_amd.load_native()
    dense = a.config == "k1024dense"
    if dense:
        w = DenseWorkload(dev, G, k, S, rank)
        engine = w.dc.engine
        a.no_host_rate = True
    else:
        w = Workload(dev, G, k, r, S, stride, m, a.mixed, rank)
        engine = w.enc.engine
    if a.mac != "auto":
        engine.set_mac_kind(a.mac)

    # optional: the HBM copy probe (reported in the roofline) before the warmup steps, with more
    # repetitions (clock ramp experiment, NTC_BENCH_PROBE_FIRST=<reps>)
    probe_reps = int(os.environ.get("NTC_BENCH_PROBE_FIRST", "0"))
    probe = hbm_copy_probe(dev, reps=probe_reps) if probe_reps else None
    nprof = min(a.steps, 10)
    step = w.step
    if a.graph:
        # the whole step (every launch of encode + decode) captured once, replayed per step: the
        # same kernels on the same buffers, only the per-launch host and dispatch cost goes
        s_cap = torch.cuda.Stream(dev)
        s_cap.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s_cap):
            for _ in range(2):
                w.step()
        torch.cuda.current_stream(dev).wait_stream(s_cap)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            w.step()
        torch.cuda.synchronize(dev)
        step = graph.replay
    engine.timing_log(nprof * 16)        # the log's events exist before the clock starts ...
    engine.timing_kinds(())              # ... but nothing is logged until the profiled steps
    # Warmup: the W steps asked for, continued (synchronised) until the device has run this load
    # for at least NTC_BENCH_MIN_WARMUP_MS (default 60): from a cold start the MI355X's clocks take
    # ~12 config-3 steps (~25 ms) to reach their steady step time (3.3 -> 1.85 ms,
    # tools/step_times.py, profiles/r04/final/step_times.txt), so at --warmup 5 a quarter of a
    # 20-step timed region would still be ramping.  The line reports both counts.
    min_warm = float(os.environ.get("NTC_BENCH_MIN_WARMUP_MS", "60")) / 1e3
    t_warm = time.perf_counter()
    warm_run = 0
    while warm_run < a.warmup or (time.perf_counter() - t_warm < min_warm and warm_run < 1000):
        step()
        warm_run += 1
        if warm_run >= a.warmup:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    barrier()
    torch.cuda.synchronize(dev)
    # the timed steps run bare: bracketing kernels with events costs 1.5 % of a config-3 step and
    # 12-15 % of a config-2 step, so `value` is measured without them
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    # graph mode: the replayed steps' own outputs are checked too (the profiled steps below run
    # eagerly, with per-launch events)
    graph_good = w.verify()[0] if a.graph else None
    # profiled steps straight after (no host work in between, so the clocks stay where the timed
    # steps left them).  (1) nprof steps with every kernel launch timed by the event pair its
    # dispatch stamps (engine timing log, hipExtLaunchKernelGGL): the kinds in a step and the
    # all-stamped breakdown.  (2) Isolated per-kernel timing: stamping every dispatch slows the
    # steps (round 4: the all-stamped decode MAC ran 2.5 % longer than rocprof's trace of the bare
    # timed steps, and the kernel sum exceeded the bare step), so each kernel kind is then timed
    # over nprof steps in which ONLY that kind carries event pairs; roofline.kernel_ms and
    # kernels_ms come from these and their sum is checked against the bare timed step.  (3) One
    # last step behind a poisoning of every output (verified below).
    engine.timing_kinds(None)
    tp = time.perf_counter()
    for _ in range(nprof):
        w.step()
    torch.cuda.synchronize(dev)
    ms_prof = (time.perf_counter() - tp) * 1e3 / nprof
    log = engine.timing_read()
    kinds_in_step = []
    for kind, _ in log:
        if kind not in kinds_in_step:
            kinds_in_step.append(kind)
    iso_log = {}
    for kind in kinds_in_step:
        engine.timing_log(nprof * 16, [kind])
        for _ in range(nprof):
            w.step()
        torch.cuda.synchronize(dev)
        iso_log[kind] = engine.timing_read()
    engine.timing_log(0)
    w.poison()
    torch.cuda.synchronize(dev)
    w.step()
    torch.cuda.synchronize(dev)
    rewritten = w.rewritten()
    # outputs of the last step (the same computation as every timed step), checked after the
    # clocks stop
    good, ndec, dec_bytes, dec_macs = w.verify()
    good = good and rewritten
    smp = w.oracle_sample() if (rank == 0 and world == 1 and not a.no_cpu_baseline) else None
    if world > 1:
        import torch.distributed as dist
        from netcode_amd.shard import max_over_ranks
        elapsed = max_over_ranks(elapsed, dist, dev)

    ms_step = elapsed / a.steps * 1e3
    payload = G * k * S * world
    value = payload / (elapsed / a.steps) / 2**30
    kern_all, launches_all = kernel_summary(log, nprof, dense)
    kern_step, launches = {}, {"encode_mac": [], "decode_mac": []}
    for kind, lg in iso_log.items():
        ks_, la_ = kernel_summary(lg, nprof, dense)
        kern_step.update(ks_)
        for n_, v_ in la_.items():
            launches[n_] += v_

    # Roofline of the dominant kernel: algorithmic bytes per launch / its mean launch duration
    # over the timed steps.  Encode MAC: read k*S, write r*S per generation; decode MAC: per
    # DECODED generation read (k-m)*S sources + m*S repairs, write m*S (singular generations get
    # no decode MAC and are not counted).
    enc_bytes = G * (k + r) * S
    t_emac = float(np.mean(launches["encode_mac"]))
    t_dmac = float(np.mean(launches["decode_mac"]))
    if t_emac >= t_dmac:
        dom, t_dom, bytes_dom, macs = "encode_mac", t_emac, enc_bytes, G * r * k * S
    else:
        dom, t_dom, bytes_dom, macs = "decode_mac", t_dmac, dec_bytes, dec_macs
    achieved = bytes_dom / (t_dom * 1e-3) / 1e9
    traffic, tsrc = pmc_record("pmc_traffic.json", a.config, dom)
    valu, vsrc = pmc_record("pmc_valu.json", a.config, dom)
    ksum = sum(kern_step.values())
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
            "traffic_source": tsrc, "kernel": dom, "kernel_ms": round(t_dom, 4),
            "kernel_ms_source": f"mean of the {len(launches[dom])} {dom} launches of {nprof} "
                                f"steps run after the timed ones in which only {dom} carries an "
                                f"event pair (stamped by its dispatch); with every launch "
                                f"stamped: {round(float(np.mean(launches_all[dom])), 4)} ms",
            "algorithmic_bytes_per_launch": int(bytes_dom),
            "byte_macs_per_launch": int(macs),
            "byte_mac_rate_T_per_s": round(macs / (t_dom * 1e-3) / 1e12, 2),
            "valu_profile": valu, "valu_profile_source": vsrc,
            "hbm_copy_probe_GBps": probe if probe is not None else hbm_copy_probe(dev)}
    if dense:
        # config 5 is compute-class: each source feeds 1024 rows, so its MACs are bound by the
        # bit-sliced chain, not HBM (0.13 GB per 0.78-ms launch).  Primary roofline: the byte-MAC
        # rate against the chain's measured ceiling; the HBM fraction stays as a secondary field.
        bm = macs / (t_dom * 1e-3) / 1e12
        hbm = {k_: roof.pop(k_) for k_ in ("achieved", "peak", "unit", "frac")}
        roof.pop("bound")
        roof = {"bound": "valu", "achieved": round(bm, 2), "peak": CHAIN_PEAK_TBMAC,
                "unit": "T byte-MAC/s", "frac": round(bm / CHAIN_PEAK_TBMAC, 4),
                "peak_source": CHAIN_PEAK_SOURCE,
                "valu_issue_frac": (valu or {}).get("valu_issue_frac"),
                "hbm_secondary": {**hbm, "note": "algorithmic bytes (k + n)*S per launch over its "
                                                 "duration, against the 8 TB/s HBM peak"},
                **roof}

    line = {"metric": metric_name(a.config, k, r, S),
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": n_gpus, "ranks": world,
            "rank_sync": backend if world > 1 else None,
            "steps": a.steps,
            "warmup": a.warmup, "warmup_steps_run": warm_run, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8 (GF(2^8))",
            "data": "synthetic (seeded random payloads, exact-m uniform loss)",
            "config": {"workload": a.config, "k": k, "r": r, "S": S, "stride": stride,
                       "m": ("U[0,%d]" % m) if a.mixed else m, "generations_per_gpu": G,
                       "parallelism": f"generation-shard x{world} (no collectives)",
                       **({"mac": a.mac} if a.mac != "auto" else {}),
                       **({"step": "HIP graph replay"} if a.graph else {})},
            "value_note": "G*k*S source-payload bytes per step over all G generations; "
                          f"{G - ndec} of {G} per rank are singular under the reference "
                          "coefficient schedule (encoded and planned, no decode MAC)",
            "value_decoded_only": round(ndec * k * S * world / (elapsed / a.steps) / 2**30, 3),
            "value_decoded_only_note": "the same step time over the payload of the generations "
                                       "that decoded only (rank 0's count x ranks)",
            "roofline": roof,
            "kernels_ms": {n: round(v, 4) for n, v in sorted(kern_step.items())},
            "kernels_ms_note": f"per step; each kernel kind timed over {nprof} steps run after "
                               f"the timed ones in which only that kind carries event pairs "
                               f"(stamped by its dispatches); the timed steps run without events",
            "kernels_ms_all_stamped": {n: round(v, 4) for n, v in sorted(kern_all.items())},
            "ms_per_step_all_stamped": round(ms_prof, 4),
            "kernel_sum_ms_per_step": round(ksum, 4),
            "kernels_fit_in_step": bool(ksum <= ms_step),
            "kernels_fit_in_stamped_step": bool(ksum <= ms_prof),
            "kernel_sum_over_step": round(ksum / ms_step, 4),
            "kernels_fit_note": "each isolated duration runs from its dispatch's start stamp to its "
                                "end stamp and so includes the kernel's own launch ramp, which in "
                                "the bare back-to-back step overlaps the previous kernel's tail: "
                                "the sum can exceed the bare step by a few us per kernel "
                                "(kernel_sum_over_step); it stays within the stamped step",
            "verified": {"decoded_generations": ndec, "bit_exact_round_trip": good,
                         "poisoned_slots_rewritten": rewritten,
                         "poison_note": "before the last step (after the profiled ones) every output (lost slots, "
                                        "repairs, encoded sizes, status) was overwritten with 0xA5; "
                                        "after it all equal the previous step's / the sources",
                         **({"graph_replay_bit_exact": graph_good} if a.graph else {})}}
    if rank == 0 and world == 1 and not a.no_host_rate:
        hk, hp, hs, hok = host_rate(w)
        line["host_resident_GiBps"] = round(hk, 3)
        line["host_resident_note"] = ("PCIe-inclusive, never `value`: sources H2D + repairs D2H, "
                                      "then only the received sources H2D and only the lost "
                                      "slots D2H (packed rows), 3 streams")
        line["host_resident_bit_exact"] = hok
        good = good and hok
        line["host_resident_full_slots_GiBps"] = round(hp, 3)
        line["host_resident_serial_GiBps"] = round(hs, 3)
        hw, hwok, rpk, rpl = host_rate_wire(w)
        line["host_resident_wire_GiBps"] = round(hw, 3)
        line["host_resident_wire_note"] = (
            "PCIe-inclusive, never `value`, socket buffer to socket buffer in the reference's wire "
            "format: sender sources H2D -> encode -> write_repairs -> repair packets D2H; receiver "
            "received source packets + repair packets H2D -> read_packets -> decode -> lost rows "
            "packed D2H; 3 streams, chunks of G/16")
        line["host_resident_wire_bit_exact"] = hwok
        if not hwok:
            line["host_resident_wire_checks"] = host_rate_wire.checks
        good = good and hwok
        if smp is not None:
            gi = torch.from_numpy(smp["g"])
            smp["rep_pkts"] = rpk.view(G, r, -1)[gi].numpy()
            smp["rep_pkt_len"] = rpl.view(G, r)[gi].numpy()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        thr = a.cpu_threads or effective_cpus()   # the CPUs this process actually gets
        line["cpu_baseline"] = (cpu_baseline_dense(w) if dense
                                else cpu_baseline(k, r, S, stride, m, thr))
        if smp is not None:
            ok, parts = oracle_check(smp, thr)
            line["verified"]["oracle_slice_bit_exact"] = ok
            line["verified"]["oracle_slice"] = {
                "generations": [int(x) for x in smp["g"]], "checked": parts,
                "how": "the bench's own last-step outputs of these generations vs or_encode_batch / "
                       "or_decode_batch on the same sources, ids and masks (cpu_baseline leg)"}
            good = good and ok
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    if not good or graph_good is False:
        sys.exit(3)


if __name__ == "__main__":
    main()
