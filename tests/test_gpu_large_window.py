"""GPU parity for large windows (m up to 255, the w = 8 limit): 64 < r <= 255
runs decode_plan_big (one workgroup per generation, Gauss-Jordan in LDS), bit-exact against the
CPU oracle's streaming decoder (detail/decoder.cc:412-566 greedy retry, :484-497 decoded sizes)
for every status outcome, under each region-MAC formulation.
"""
import numpy as np
import pytest

from helpers import loss_exact_m, loss_mixed_m, make_sources
from oracle import oracle as O
from test_gpu_parity import gpu_decode, gpu_encode, mac  # noqa: F401  (mac is a fixture)

pytestmark = pytest.mark.gpu


def run_case(d, G, k, r, S, stride, mask, rmask, seed, ids=False):
    src, lens = make_sources(G, k, S, stride, seed=seed, ragged=True)
    sid = rid = None
    if ids:
        rng = np.random.default_rng(seed + 5)
        sid = rng.integers(0, 2**32 - 70000, G, dtype=np.uint64).astype(np.uint32)
        rid = rng.integers(0, 2**32 - 70000, G, dtype=np.uint64).astype(np.uint32)
    rep, rsz, _ = gpu_encode(d, src, lens, k, r, sid, rid)
    orep, orsz = O.encode_batch(src, lens, k, r, sid, rid)
    assert (rep == orep).all(), "encode mismatch"
    assert (rsz == orsz).all()
    lost = src.copy()
    lost[mask == 0] = 0
    llen = lens.copy()
    llen[mask == 0] = 0
    out, olen_gpu, st = gpu_decode(d, lost, llen, mask, rep, rsz, rmask, sid, rid)
    oout, olen, ost = O.decode_batch(lost, llen, mask, orep, orsz, rmask, sid, rid)
    assert (st == ost).all(), f"status mismatch\n{st}\n{ost}"
    assert (olen_gpu == olen).all(), "decoded sizes mismatch"
    assert (out == oout).all(), "payload mismatch"
    return ost


# (300, 100, 80): with the reference's coefficient schedule every candidate matrix of these
# generations is singular (state 3, 21 failed attempts each, as the oracle reports); (300, 100, 40)
# mixes one such generation with decoded ones.
@pytest.mark.parametrize("k,r,m,stride,decoded", [(300, 100, 40, 256, 2), (300, 100, 80, 256, 0),
                                                  (200, 65, 65, 64, 3), (160, 128, 97, 2048, 3)])
def test_large_window_exact_loss(gpu, mac, k, r, m, stride, decoded):
    G = 3
    mask = loss_exact_m(G, k, m, seed=k + r)
    st = run_case(gpu, G, k, r, stride, stride, mask, np.ones((G, r), np.uint8), seed=r)
    assert int((st["state"] == 0).sum()) == decoded


def test_large_window_r255_mixed(gpu, mac):
    """r = 255 with mixed losses up to r, lost repairs, explicit id bases: decoded, not enough
    repairs, nothing missing and (rarely) singular outcomes all match the oracle."""
    G, k, r, stride = 6, 300, 255, 128
    mask = loss_mixed_m(G, k, r, seed=11)
    mask[0] = 1                                    # nothing missing
    rmask = (np.random.default_rng(12).random((G, r)) > 0.05).astype(np.uint8)
    rmask[1, :] = 0                                # not enough repairs
    st = run_case(gpu, G, k, r, stride, stride, mask, rmask, seed=13, ids=True)
    assert st["state"][0] == 1 and st["state"][1] == 2


def test_decode_rejects_r_over_255(gpu):
    import torch
    from netcode_amd import BatchDecoder, NativeError
    G, k, r, S = 1, 8, 256, 64
    t = lambda *s, dt=torch.uint8: torch.zeros(s, dtype=dt, device=gpu)
    with pytest.raises(NativeError):
        BatchDecoder(k, r, gpu)(t(G, k, S), t(G, k, dt=torch.int16), t(G, k), t(G, r, S),
                                t(G, r, dt=torch.int16), t(G, r))
