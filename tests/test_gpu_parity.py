"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle, bit-exact.

Reference behaviour covered: detail/encoder.cc:15-64 (repairs, encoded sizes, zero padding of
shorter sources), detail/decoder.cc:54-152 + 412-566 (reduction, peeling, full decoding, greedy
drop of the newest repair on a singular matrix, useless repairs), galois_field.hh:65-158.
"""
import os

import numpy as np
import pytest

from helpers import loss_exact_m, loss_iid, loss_mixed_m, make_sources

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def dev(a, d):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    elif a.dtype == np.uint32:
        a = a.view(np.int32)
    return torch.from_numpy(a.copy()).to(d)


def host(t, dtype=None):
    a = t.cpu().numpy()
    return a.view(dtype) if dtype is not None else a


def gpu_encode(d, src, lens, k, r, sid=None, rid=None):
    from netcode_amd import BatchEncoder
    res = BatchEncoder(k, r, d)(dev(src, d), dev(lens, d),
                                None if sid is None else dev(sid, d),
                                None if rid is None else dev(rid, d))
    return host(res.repairs), host(res.encoded_size, np.uint16), host(res.symbol_len, np.uint16)


def gpu_decode(d, lost, llen, smask, rep, rsz, rmask, sid=None, rid=None):
    import torch
    from netcode_amd import BatchDecoder, status_to_numpy
    k, r = lost.shape[1], rep.shape[1]
    s_t, l_t = dev(lost, d), dev(llen, d)
    st = BatchDecoder(k, r, d)(s_t, l_t, dev(smask, d), dev(rep, d), dev(rsz, d), dev(rmask, d),
                               None if sid is None else dev(sid, d),
                               None if rid is None else dev(rid, d))
    torch.cuda.synchronize(d)
    return host(s_t), host(l_t, np.uint16), status_to_numpy(st)


@pytest.fixture(params=["auto", "perm", "bitslice", "grouped", "paired"])
def mac(request, gpu):
    """Run a parity test under each region-MAC formulation (ntc_gf256_set_mac_kind)."""
    from netcode_amd.engine import Engine
    eng = Engine.get(gpu)
    eng.set_mac_kind(request.param)
    yield request.param
    eng.set_mac_kind("auto")


def test_region_multiply(gpu, oracle):
    import torch
    from netcode_amd import GaloisField
    gf = GaloisField(8, gpu)
    rng = np.random.default_rng(1)
    L = oracle.lib()
    for n in [1, 3, 4, 17, 1024, 1500, 65535]:
        src = rng.integers(0, 256, n, dtype=np.uint8)
        dst0 = rng.integers(0, 256, n, dtype=np.uint8)
        for c in [0, 1, 2, 0x53, 255]:
            for add in (0, 1):
                s_t, d_t = dev(src, gpu), dev(dst0, gpu)
                (gf.multiply_add if add else gf.multiply)(s_t, d_t, n, c)
                torch.cuda.synchronize()
                ref = dst0.copy()
                (L.or_region_muladd if add else L.or_region_mul)(oracle._p(src), oracle._p(ref), n, c)
                assert (host(d_t) == ref).all(), (n, c, add)


ENCODE_CASES = [
    # G, k, r, S, stride, ragged, id_mode
    (64, 32, 8, 1024, 1024, False, "default"),        # config 2 shape
    (8, 128, 32, 4096, 4096, False, "default"),       # config 3 shape
    (8, 128, 32, 1500, 1504, False, "wrap"),          # config 4 shape, uint32 wraparound ids
    (16, 16, 4, 1024, 1024, True, "offset"),          # config 1 generation form, ragged
    (8, 20, 5, 64, 64, True, "offset"),               # r not a multiple of the row tile
    (4, 33, 40, 256, 256, False, "offset"),           # odd k, r > 32 (two row chunks)
    (3, 1, 1, 16, 16, True, "default"),               # minimum shape
    (2, 7, 3, 4096, 4112, True, "offset"),            # stride not a multiple of the wave span
    (5, 9, 12, 2080, 2080, True, "offset"),           # 2 KiB spans + a 1-lane tail; 8+4 row tiles
    (6, 21, 20, 2048, 2048, False, "offset"),         # 3 row tiles: plane-sharing group, one idle wave
    # lean-loop MAC (full 2 KiB spans, k % 4 == 0): only the final group of 4 sources; 3 spans
    (5, 4, 3, 2048, 2048, True, "offset"),
    (3, 12, 9, 6144, 6144, True, "wrap"),
    # split-k (few tasks, k >= 128): parts of 68 sources and a short last part, partial outputs
    # XORed by ksplit_reduce; ragged spans, 16 + 4 row tiles
    (2, 203, 20, 2080, 2080, True, "offset"),
    (3, 130, 17, 4096, 4096, False, "wrap"),
    # generation pairing (continuous ids, stride <= 1024, G > 255): g and g + 255 share one MAC
    # wave when their matrices match; a tail of unpaired generations; odd row tiles; half fill
    (700, 32, 8, 1024, 1024, True, "default"),
    (600, 16, 4, 512, 512, True, "default"),
    (520, 9, 20, 688, 688, True, "default"),
    (600, 16, 4, 1024, 1024, False, "offset"),        # explicit continuous bases
    (600, 16, 4, 1024, 1024, False, "wrap"),          # explicit bases whose products wrap
    # config 2 itself: uint32 wraps make some g / g + 255 matrices differ (those stay unpaired)
    (4096, 32, 8, 1024, 1024, False, "default"),
    # r > 256: encode_prep walks the coefficients in chunks of 256 rows (two chunks here, the
    # second ragged); uint32-wrapping ids and unequal lengths (one size product per source)
    (3, 37, 300, 1024, 1024, True, "wrap"),
    (2, 64, 513, 512, 512, False, "offset"),
    # >= 384 rows over whole 2 KiB spans: sources pre-sliced once (bs_preslice + the SL MAC); a
    # ragged last row tile, and split-k parts reading the sliced copy
    (2, 37, 400, 2048, 2048, True, "wrap"),
    (1, 130, 390, 4096, 4096, False, "offset"),
    (2, 128, 400, 2048, 2048, True, "default"),       # two generations' parts in one sliced copy
    # tile-pair workgroups (gf_mac_bsg, > 16 rows): k below the group size (wave 1 builds no
    # source, or one), partial spans with a short k, a second group with one idle wave
    (4, 1, 24, 2048, 2048, True, "offset"),
    (3, 2, 17, 4096, 4096, False, "default"),
    (3, 3, 40, 4112, 4112, True, "offset"),
    (2, 5, 33, 2080, 2080, True, "wrap"),
]


def _ids(mode, G, k, r):
    if mode == "default":
        return None, None
    if mode == "offset":
        return ((np.arange(G) * k + 11).astype(np.uint32), (np.arange(G) * r + 5).astype(np.uint32))
    # config 4: continuous ids of a 65536-generation run; rid*sid products exceed 2^32
    base = 65536 - G
    return (((base + np.arange(G)) * k).astype(np.uint32), ((base + np.arange(G)) * r).astype(np.uint32))


@pytest.mark.parametrize("G,k,r,S,stride,ragged,ids", ENCODE_CASES)
def test_encode_parity(gpu, mac, oracle, G, k, r, S, stride, ragged, ids):
    src, lens = make_sources(G, k, S, stride, seed=G * 1000 + k + r, ragged=ragged)
    sid, rid = _ids(ids, G, k, r)
    rep, rsz, rlen = gpu_encode(gpu, src, lens, k, r, sid, rid)
    orep, orsz = oracle.encode_batch(src, lens, k, r, sid, rid)
    assert (rsz == orsz).all()
    assert (rlen == lens.max(axis=1)).all()
    assert (rep == orep).all()


@pytest.mark.parametrize("name", ["gen_k16_r4_loss25", "gen_k32_r8_ragged"])
def test_decode_golden_fixtures(gpu, mac, name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"))
    k, r = z["src"].shape[1], z["rep"].shape[1]
    rep, rsz, _ = gpu_encode(gpu, z["src"], z["src_len"], k, r, z["sid_base"], z["rid_base"])
    assert (rep == z["rep"]).all() and (rsz == z["rep_size"]).all()
    lost = z["src"].copy()
    lost[z["src_mask"] == 0] = 0
    llen = z["src_len"].copy()
    llen[z["src_mask"] == 0] = 0
    out, olen, st = gpu_decode(gpu, lost, llen, z["src_mask"], rep, rsz, z["rep_mask"],
                               z["sid_base"], z["rid_base"])
    assert (st.view(np.uint8).reshape(len(st), -1) == z["status"]).all()
    assert (olen == z["out_len"]).all()
    assert (out == z["out"]).all()


DECODE_CASES = [
    # G, k, r, S, stride, loss kind, param, ragged
    (64, 32, 8, 1024, 1024, "exact", 8, False),       # config 2
    (6, 128, 32, 4096, 4096, "exact", 32, False),     # config 3 worst case
    (24, 128, 32, 4096, 4096, "mixed", 32, False),    # config 3 mixed m ~ U[0,32]
    (8, 128, 32, 1500, 1504, "exact", 31, True),      # config 4 shape
    (200, 16, 4, 1024, 1024, "iid", 0.25, False),     # config 1 generation form (singulars)
    (40, 32, 8, 512, 512, "exact", 1, True),          # single loss -> peeling path
    (40, 32, 8, 512, 512, "exact", 0, False),         # nothing missing -> useless repairs
    (10, 48, 40, 256, 256, "exact", 40, False),       # m = r = 40 (> one row tile)
    (9, 33, 12, 2080, 2080, "exact", 12, True),       # odd k (unaligned plan rows), 8+4 row tiles
    (30, 7, 5, 4096, 4096, "iid", 0.3, False),        # tiny k, mixed outcomes
    (12, 45, 24, 2048, 2048, "mixed", 24, False),     # k % 4 != 0, 1-3 row tiles per generation
    (20, 8, 8, 2048, 2048, "iid", 0.3, True),         # lean-loop MAC: k = 8 (two groups of 4)
    (7, 12, 16, 6144, 6144, "exact", 9, False),       # lean-loop MAC: 3 spans, 8+1 row tiles
    # iid loss of sources and repairs, r > 32: a few generations decode only after the first
    # candidate repair fails (decoder.cc:448-468 retry; the LDS plan's rank screening)
    (400, 100, 64, 64, 64, "iid", 0.35, False),
    (400, 60, 40, 64, 64, "iid", 0.3, True),
    # tile-pair workgroups (gf_mac_bsg): m ~ U[0, 20] (some pairs with an idle second wave, some
    # generations with nothing to decode), and 3 row tiles over a partial span
    (16, 24, 20, 2048, 2048, "mixed", 20, True),
    (10, 40, 36, 4112, 4112, "exact", 36, False),
]


@pytest.mark.parametrize("G,k,r,S,stride,kind,param,ragged", DECODE_CASES)
def test_decode_parity(gpu, mac, oracle, G, k, r, S, stride, kind, param, ragged):
    seed = G * 7 + k * 3 + r
    src, lens = make_sources(G, k, S, stride, seed=seed, ragged=ragged)
    sid = (np.arange(G) * k + 3).astype(np.uint32)
    rid = (np.arange(G) * r + 9).astype(np.uint32)
    rep, rsz, _ = gpu_encode(gpu, src, lens, k, r, sid, rid)
    if kind == "exact":
        smask = loss_exact_m(G, k, param, seed + 1)
        rmask = np.ones((G, r), np.uint8)
    elif kind == "mixed":
        smask = loss_mixed_m(G, k, param, seed + 1)
        rmask = np.ones((G, r), np.uint8)
    else:
        smask = loss_iid((G, k), param, seed + 1)
        rmask = loss_iid((G, r), param, seed + 2)
    lost = src.copy()
    lost[smask == 0] = 0
    llen = lens.copy()
    llen[smask == 0] = 0
    out, olen, st = gpu_decode(gpu, lost, llen, smask, rep, rsz, rmask, sid, rid)
    oout, oolen, ost = oracle.decode_batch(lost, llen, smask, rep, rsz, rmask, sid, rid)
    assert (st == ost).all(), (st[st != ost][:4], ost[st != ost][:4])
    assert (olen == oolen).all()
    assert (out == oout).all()
    ok = st["state"] == 0
    assert (out[ok] == src[ok]).all()


@pytest.mark.parametrize("plan", ["wave", "lds", "big"])
@pytest.mark.parametrize("G,k,r,S,stride,kind,param,ragged", DECODE_CASES)
def test_decode_parity_plan_kinds(gpu, oracle, plan, G, k, r, S, stride, kind, param, ragged):
    """Every decode-plan kernel (ntc_gf256_set_plan_kind) on every decode case: the register
    wave plan (r <= 32, else the LDS plan), the LDS wave plan (r <= 64) and the workgroup plan
    with rank screening (decode_plan_big, forced for small r too) give the oracle's bytes,
    sizes and status."""
    from netcode_amd.engine import Engine
    eng = Engine.get(gpu)
    eng.set_plan_kind(plan)
    try:
        test_decode_parity(gpu, "auto", oracle, G, k, r, S, stride, kind, param, ragged)
    finally:
        eng.set_plan_kind("auto")


def test_kernel_timing_log(gpu):
    """ntc_gf256_timing_log / timing_read (bench.py's in-step kernel clock): one entry per launch
    in launch order, positive durations whose sum fits inside the calls' wall time."""
    import torch
    from netcode_amd import BatchDecoder, BatchEncoder
    from netcode_amd.engine import Engine
    G, k, r, S = 64, 64, 16, 4096
    src, lens = make_sources(G, k, S, S, seed=3)
    s_t, l_t = dev(src, gpu), dev(lens, gpu)
    eng = Engine.get(gpu)
    smask = dev(loss_exact_m(G, k, 8, 4), gpu)
    rmask = torch.ones((G, r), dtype=torch.uint8, device=gpu)
    enc = BatchEncoder(k, r, gpu)(s_t, l_t)
    torch.cuda.synchronize(gpu)
    eng.timing_log(64)
    try:
        s = torch.cuda.current_stream(gpu)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        enc = BatchEncoder(k, r, gpu)(s_t, l_t, out=enc)
        BatchDecoder(k, r, gpu)(s_t, l_t, smask, enc.repairs, enc.encoded_size, rmask)
        ev[1].record(s)
        log = eng.timing_read()
        torch.cuda.synchronize(gpu)
        names = [n for n, _ in log]
        assert names[0] == "encode_prep" and names[-1] == "decode_mac"
        assert names.index("encode_mac") < names.index("decode_plan")
        assert all(ms > 0 for _, ms in log)
        assert sum(ms for _, ms in log) <= ev[0].elapsed_time(ev[1]) + 1e-3
    finally:
        eng.timing_log(0)


def test_full_size_round_trip_config3(gpu, oracle):
    """Config 3 at BASELINE size (G=4096, k=128, r=32, 4 KiB, m=32).  Size-independent checks:
    every generation the plan reports decoded reproduces its sources exactly, and the per-
    generation outcome (which matrices are singular under the reference coefficient schedule,
    ~2 % here) equals the oracle's, which depends only on ids and loss pattern."""
    import torch
    from netcode_amd import BatchDecoder, BatchEncoder, status_to_numpy
    G, k, r, S = 4096, 128, 32, 4096
    g = torch.Generator(device=gpu).manual_seed(5)
    src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=gpu, generator=g)
    lens = torch.full((G, k), S, dtype=torch.int16, device=gpu)
    enc = BatchEncoder(k, r, gpu)(src, lens)
    mask = loss_exact_m(G, k, 32, seed=6)
    smask = torch.from_numpy(mask).to(gpu)
    lost = src * smask[:, :, None]
    llen = lens * smask.to(torch.int16)
    st = status_to_numpy(BatchDecoder(k, r, gpu)(lost, llen, smask, enc.repairs, enc.encoded_size,
                                                 torch.ones((G, r), dtype=torch.uint8, device=gpu)))
    ok = torch.from_numpy(st["state"] == 0).to(gpu)
    assert bool((lost[ok] == src[ok]).all())
    assert bool((llen[ok] == lens[ok]).all())
    # outcome parity with the oracle on a 16-byte slice of the same generations
    s16 = src[:, :, :16].cpu().numpy()
    l16 = np.full((G, k), 16, np.uint16)
    orep, orsz = oracle.encode_batch(s16, l16, k, r, threads=16)
    _, _, ost = oracle.decode_batch(s16 * mask[:, :, None], l16 * mask, mask, orep, orsz,
                                    np.ones((G, r), np.uint8), threads=16)
    assert (st == ost).all()


def test_mac_timing_api(gpu):
    """ntc_gf256_set_timing / mac_time (the bench's roofline clock): the recorded MAC durations
    are positive and no longer than the whole encode / decode call around them."""
    import ctypes as C
    import torch
    from netcode_amd import BatchDecoder, BatchEncoder, _native
    from netcode_amd.engine import Engine
    G, k, r, S = 64, 64, 16, 4096
    src, lens = make_sources(G, k, S, S, seed=3)
    s_t, l_t = dev(src, gpu), dev(lens, gpu)
    L, h = _native.load(), Engine.get(gpu).handle
    _native.check(L.ntc_gf256_set_timing(h, 1), "timing")
    try:
        s = torch.cuda.current_stream(gpu)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        enc = BatchEncoder(k, r, gpu)(s_t, l_t)
        ev[1].record(s)
        torch.cuda.synchronize()
        ms = C.c_float()
        _native.check(L.ntc_gf256_mac_time(h, 0, C.byref(ms)), "mac time")
        assert 0 < ms.value <= ev[0].elapsed_time(ev[1]) + 1e-3
        smask = loss_exact_m(G, k, 8, 4)
        BatchDecoder(k, r, gpu)(s_t, l_t, dev(smask, gpu), enc.repairs, enc.encoded_size,
                                torch.ones((G, r), dtype=torch.uint8, device=gpu))
        _native.check(L.ntc_gf256_mac_time(h, 1, C.byref(ms)), "mac time")
        assert ms.value > 0
    finally:
        _native.check(L.ntc_gf256_set_timing(h, 0), "timing")


def test_decode_apply_after_other_buffers(gpu, oracle):
    """decode_batch(A, B) leaves the decode MAC's input row addresses of A / B in the engine (the
    register plan writes them); decode_apply on other buffers C / D overwrites them (plan_rows),
    so a later decode_apply(A, B) must not reuse them (advisor r2: a stale row cache read C / D).
    The last apply must equal the oracle's decode of A / B."""
    import torch
    from netcode_amd import BatchDecoder, _native
    from netcode_amd.engine import Engine, _stream
    G, k, r, S, m = 16, 64, 16, 4096, 12
    src, lens = make_sources(G, k, S, S, seed=41)
    rep, rsz, _ = gpu_encode(gpu, src, lens, k, r)
    smask = loss_exact_m(G, k, m, seed=42)
    rmask = np.ones((G, r), np.uint8)
    lost = src.copy()
    lost[smask == 0] = 0
    llen = lens.copy()
    llen[smask == 0] = 0
    oout, oolen, ost = oracle.decode_batch(lost, llen, smask, rep, rsz, rmask)
    A, B = dev(lost, gpu), dev(rep, gpu)
    BatchDecoder(k, r, gpu)(A, dev(llen, gpu), dev(smask, gpu), B, dev(rsz, gpu), dev(rmask, gpu))
    torch.cuda.synchronize(gpu)
    assert (host(A) == oout).all()
    rng = np.random.default_rng(43)
    C = dev(rng.integers(0, 256, lost.shape, dtype=np.uint8), gpu)
    D = dev(rng.integers(0, 256, rep.shape, dtype=np.uint8), gpu)
    L, h, st = _native.load(), Engine.get(gpu).handle, _stream(gpu)
    _native.check(L.ntc_gf256_decode_apply(h, G, k, r, S, C.data_ptr(), D.data_ptr(), st), "apply C/D")
    A.copy_(dev(lost, gpu))
    _native.check(L.ntc_gf256_decode_apply(h, G, k, r, S, A.data_ptr(), B.data_ptr(), st), "apply A/B")
    torch.cuda.synchronize(gpu)
    assert (host(A) == oout).all()
