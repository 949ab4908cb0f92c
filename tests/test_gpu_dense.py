"""GPU parity for dense codes (BASELINE config 5 extension): device Gauss-Jordan inversion,
dense encode and decode against the CPU oracle (or_invert = the reference's jerasure-order
detail::invert, invert_matrix.cc:9-128, plus region MACs), bit-exact.

The reference has no dense large-k path (its w = 8 schedule is singular beyond 255 sources), so
the oracle here is its own inversion routine applied to caller-chosen matrices.  At the full
config-5 size (k = 1024, 64 KiB symbols) parity is checked by the encode -> decode round trip.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _dev(a, d):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).copy()).to(d)


def _mats(G, n, seed, singular=()):
    rng = np.random.default_rng(seed)
    mats = rng.integers(0, 256, (G, n, n), dtype=np.uint8)
    for g in singular:
        if n >= 2:
            mats[g, n - 1] = mats[g, 0] ^ mats[g, n // 2] if n > 2 else mats[g, 0]
        else:
            mats[g, 0, 0] = 0
    return mats


@pytest.mark.parametrize("n", [1, 2, 5, 31, 32, 33, 64, 100, 256])
def test_dense_invert(gpu, oracle, n):
    import torch
    from netcode_amd import DenseCode
    G = 4
    mats = _mats(G, n, seed=n, singular=(2,))
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, (n, g)
        assert (inv[g] == o_inv).all(), (n, g)


def test_dense_invert_many_generations(gpu, oracle):
    """Many generations per launch: the lookahead launches (dn_fused) run one panel block per
    generation ahead of the update blocks; two singular generations among them."""
    import torch
    from netcode_amd import DenseCode
    G, n = 40, 96
    mats = _mats(G, n, seed=11, singular=(7, 31))
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, g
        assert (inv[g] == o_inv).all(), g


def test_dense_invert_structured(gpu, oracle):
    """Zero pivots that force row exchanges, identity, permutation, all-zero matrices."""
    import torch
    from netcode_amd import DenseCode
    n = 64
    rng = np.random.default_rng(5)
    perm = np.zeros((n, n), np.uint8)
    perm[np.arange(n), rng.permutation(n)] = rng.integers(1, 256, n, dtype=np.uint8)
    lower = np.tril(rng.integers(0, 256, (n, n), dtype=np.uint8), -1)
    lower[np.arange(n), np.arange(n)] = 0          # zero diagonal: every pivot needs a swap
    lower[0, n - 1] = 7
    mats = np.stack([np.eye(n, dtype=np.uint8), perm, lower, np.zeros((n, n), np.uint8)])
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(len(mats)):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, g
        assert (inv[g] == o_inv).all(), g


@pytest.mark.parametrize("n,density", [(256, 0.02), (300, 0.05), (512, 0.01)])
def test_dense_invert_sparse(gpu, oracle, n, density):
    """Sparse matrices: the owner wave often has no candidate (fallback election), rows of many
    waves become pivots out of order; some of these matrices are singular."""
    import torch
    from netcode_amd import DenseCode
    G = 3
    rng = np.random.default_rng(n)
    vals = rng.integers(1, 256, (G, n, n), dtype=np.uint8)
    mats = np.where(rng.random((G, n, n)) < density, vals, 0).astype(np.uint8)
    for g in range(G):           # a random permutation with non-zero entries keeps most invertible
        mats[g, np.arange(n), rng.permutation(n)] = rng.integers(1, 256, n, dtype=np.uint8)
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, (n, g)
        assert (inv[g] == o_inv).all(), (n, g)


@pytest.mark.parametrize("G,n,k,S", [(3, 40, 40, 1024), (2, 128, 128, 4096), (1, 200, 200, 1504)])
def test_dense_encode_decode(gpu, oracle, G, n, k, S):
    import torch
    from netcode_amd import DenseCode
    dc = DenseCode(gpu)
    rng = np.random.default_rng(G * 1000 + n)
    src = rng.integers(0, 256, (G, k, S), dtype=np.uint8)
    mats = _mats(G, n, seed=S, singular=(G - 1,) if G > 1 else ())
    rep = dc.encode(_dev(mats, gpu), _dev(src, gpu))
    out, ok = dc.decode(_dev(mats, gpu), rep)
    torch.cuda.synchronize(gpu)
    rep, out, ok = rep.cpu().numpy(), out.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        assert (rep[g] == oracle.dense_encode(mats[g], src[g])).all(), g
        o_ok, o_out, _ = oracle.dense_decode(mats[g], rep[g])
        assert bool(ok[g]) == o_ok
        assert (out[g] == o_out).all(), g
        if o_ok:
            assert (out[g] == src[g]).all()


def test_dense_inverse_512_exact(gpu, oracle):
    import torch
    from netcode_amd import DenseCode
    mats = _mats(1, 512, seed=512)
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    o_ok, _, o_inv = oracle.dense_decode(mats[0], np.zeros((512, 16), np.uint8))
    assert o_ok and bool(ok.cpu().numpy()[0])
    assert (inv.cpu().numpy()[0] == o_inv).all()


def test_dense_config5_round_trip(gpu):
    """BASELINE config 5 at full size: k = 1024 all lost, 1024 dense repairs, 64 KiB symbols."""
    import torch
    from netcode_amd import DenseCode
    dc = DenseCode(gpu)
    k, S = 1024, 65536
    g = torch.Generator(device=gpu).manual_seed(5)
    src = torch.randint(0, 256, (1, k, S), dtype=torch.uint8, device=gpu, generator=g)
    mat = torch.randint(0, 256, (1, k, k), dtype=torch.uint8, device=gpu, generator=g)
    rep = dc.encode(mat, src)
    out, ok = dc.decode(mat, rep)
    torch.cuda.synchronize(gpu)
    assert int(ok.item()) == 1
    assert torch.equal(out, src)


def test_dense_invert_xor_derivation_sizes(gpu, oracle):
    """The 8-wave lookahead derivation (ds_xor accumulation) with a ragged last wave (n = 480:
    rows 480-511 of the block are padding) and a singular generation among three."""
    import torch
    from netcode_amd import DenseCode
    G, n = 3, 480
    mats = _mats(G, n, seed=480, singular=(1,))
    inv, ok = DenseCode(gpu).invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, g
        assert (inv[g] == o_inv).all(), g


def test_dense_round_trip_16_waves_two_generations(gpu):
    """The 16-wave derivation (n = 1000, padded to 1024) for two generations, one singular: the
    invertible one round-trips, the singular one is reported as such."""
    import torch
    from netcode_amd import DenseCode
    dc = DenseCode(gpu)
    G, k, S = 2, 1000, 1024
    g = torch.Generator(device=gpu).manual_seed(6)
    src = torch.randint(0, 256, (G, k, S), dtype=torch.uint8, device=gpu, generator=g)
    mats = _mats(G, k, seed=1000, singular=(1,))
    mat = _dev(mats, gpu)
    rep = dc.encode(mat, src)
    out, ok = dc.decode(mat, rep)
    torch.cuda.synchronize(gpu)
    assert ok.cpu().numpy().tolist() == [1, 0]
    assert torch.equal(out[0], src[0])


def test_dense_invert_stale_pivots_after_large_invert(gpu, oracle):
    """the lookahead panel reads the previous panel's pivots before it knows
    whether the generation is still live.  A large inversion first leaves pivot indices up to
    n - 1 = 767 in the engine's workspace; the many-generation inversion that follows has
    generations singular from the first column (never write a pivot) and singular later (stop
    writing them), whose stale entries must not be used as row indices."""
    import torch
    from netcode_amd import DenseCode
    dc = DenseCode(gpu)
    big = _mats(1, 768, seed=768)
    inv, ok = dc.invert(_dev(big, gpu))
    torch.cuda.synchronize(gpu)
    assert int(ok.cpu().numpy()[0]) == 1
    G, n = 48, 96
    mats = _mats(G, n, seed=96, singular=(3, 20, 47))
    mats[5, :, 0] = 0                      # singular at the very first column
    mats[30, :, :40] = 0                   # singular in the second panel
    mats[30, np.arange(32), np.arange(32)] = 1
    inv, ok = dc.invert(_dev(mats, gpu))
    torch.cuda.synchronize(gpu)
    inv, ok = inv.cpu().numpy(), ok.cpu().numpy()
    for g in range(G):
        o_ok, _, o_inv = oracle.dense_decode(mats[g], np.zeros((n, 16), np.uint8))
        assert bool(ok[g]) == o_ok, g
        assert (inv[g] == o_inv).all(), g
    assert not ok[5] and not ok[30] and not ok[3]
