"""GPU parity over seeded random shapes: encode + decode through the C ABI against the CPU oracle.

The hand-picked cases of test_gpu_parity.py pin the paths one at a time; this sweep draws
(G, k, r, S, stride, id bases, loss model, ragged lengths) at random, so row-tile / span / split-k
/ pairing / plan-kind boundaries are crossed in combinations nobody listed.  The reference
behaviour is the same (detail/encoder.cc:15-64, detail/decoder.cc:54-152 + 412-566,
galois_field.hh:65-158); each case stays under ~4 MB of payload so the oracle finishes in
well under a second.
"""
import numpy as np
import pytest

from helpers import loss_exact_m, loss_iid, loss_mixed_m, make_sources
from test_gpu_parity import gpu_decode, gpu_encode

pytestmark = pytest.mark.gpu

N_CASES = 120


def draw(seed):
    rng = np.random.default_rng(1000 + seed)
    k = int(rng.choice([1, 2, 3, 5, 8, 16, 31, 32, 33, 64, 100, 128, 130, 160, 203, 256]))
    r = int(rng.choice([1, 2, 4, 7, 8, 9, 16, 17, 24, 32]))
    S = int(rng.choice([16, 48, 300, 512, 1000, 1024, 1500, 2048, 2080, 4096, 5000]))
    stride = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    budget = 4 << 20
    G = max(1, min(int(rng.integers(1, 600)), budget // (k * stride)))
    ids = str(rng.choice(["default", "offset", "wrap", "sparse"]))
    kind = str(rng.choice(["exact", "mixed", "iid"]))
    ragged = bool(rng.integers(0, 2))
    return G, k, r, S, stride, ids, kind, ragged, rng


def id_bases(mode, G, k, r, rng):
    if mode == "default":
        return None, None
    if mode == "offset":
        return ((np.arange(G) * k + 5).astype(np.uint32), (np.arange(G) * r + 11).astype(np.uint32))
    if mode == "wrap":      # uint32 id wraparound at a generation boundary inside the batch
        h = G // 2
        return (((np.arange(G, dtype=np.int64) - h) * k % 2**32).astype(np.uint32),
                ((np.arange(G, dtype=np.int64) - h) * r % 2**32).astype(np.uint32))
    # sparse: independent random bases (no pairing congruence); ids must not wrap inside one
    # generation (include/netcode/gpu.h)
    return (rng.integers(0, 2**32 - k, G, dtype=np.int64).astype(np.uint32),
            rng.integers(0, 2**32 - r, G, dtype=np.int64).astype(np.uint32))


@pytest.mark.parametrize("case", range(N_CASES))
def test_random_shape_round_trip(gpu, oracle, case):
    G, k, r, S, stride, ids, kind, ragged, rng = draw(case)
    src, lens = make_sources(G, k, S, stride, seed=77 + case, ragged=ragged)
    sid, rid = id_bases(ids, G, k, r, rng)
    rep, rsz, rlen = gpu_encode(gpu, src, lens, k, r, sid, rid)
    orep, orsz = oracle.encode_batch(src, lens, k, r, sid, rid)
    shape = dict(G=G, k=k, r=r, S=S, stride=stride, ids=ids, kind=kind, ragged=ragged)
    assert (rsz == orsz).all(), shape
    assert (rlen == lens.max(axis=1)).all(), shape
    assert (rep == orep).all(), shape
    m = min(k, r)
    if kind == "exact":
        smask = loss_exact_m(G, k, int(rng.integers(0, m + 1)), 5 + case)
        rmask = np.ones((G, r), np.uint8)
    elif kind == "mixed":
        smask = loss_mixed_m(G, k, m, 5 + case)
        rmask = np.ones((G, r), np.uint8)
    else:
        smask = loss_iid((G, k), float(rng.uniform(0.05, 0.4)), 5 + case)
        rmask = loss_iid((G, r), float(rng.uniform(0.0, 0.3)), 6 + case)
    lost = src.copy()
    lost[smask == 0] = 0
    llen = lens.copy()
    llen[smask == 0] = 0
    if sid is None:
        sid = (np.arange(G) * k).astype(np.uint32)
        rid = (np.arange(G) * r).astype(np.uint32)
    out, olen, st = gpu_decode(gpu, lost, llen, smask, rep, rsz, rmask, sid, rid)
    oout, oolen, ost = oracle.decode_batch(lost, llen, smask, rep, rsz, rmask, sid, rid)
    bad = np.nonzero(st != ost)[0]
    assert bad.size == 0, (shape, bad[:4].tolist(), st[bad[:4]].tolist(), ost[bad[:4]].tolist())
    assert (olen == oolen).all(), shape
    assert (out == oout).all(), shape
    ok = st["state"] == 0
    assert (out[ok] == src[ok]).all(), shape
