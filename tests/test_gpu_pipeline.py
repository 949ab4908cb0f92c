"""GPU: the host-resident HostPipeline (pinned host buffers streamed through several HIP streams in
chunks of generations) gives byte-identical repairs, recovered sources and status to the CPU
oracle, for ragged chunks, explicit id bases and every entry point (encode, decode,
encode_decode).  Reference behaviour: detail/encoder.cc:15-64, detail/decoder.cc:412-566.
"""
import numpy as np
import pytest

from helpers import loss_mixed_m, make_sources
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def pinned(a):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint16:
        a = a.view(np.int16)
    return torch.from_numpy(a.copy()).pin_memory()


def case(G, k, r, S, seed, explicit_ids=True):
    src, lens = make_sources(G, k, S, S, seed=seed, ragged=True)
    mask = loss_mixed_m(G, k, r, seed=seed + 1)
    rmask = (np.random.default_rng(seed + 2).random((G, r)) > 0.1).astype(np.uint8)
    rng = np.random.default_rng(seed + 3)
    sid = rng.integers(0, 2**32 - 4096, G, dtype=np.uint64).astype(np.uint32)
    rid = rng.integers(0, 2**32 - 4096, G, dtype=np.uint64).astype(np.uint32)
    if not explicit_ids:
        sid = rid = None          # the oracle's (and the kernels') defaults g*k / g*r
    orep, orsz = O.encode_batch(src, lens, k, r, sid, rid)
    lost = src.copy()
    lost[mask == 0] = 0
    llen = lens.copy()
    llen[mask == 0] = 0
    oout, olen, ost = O.decode_batch(lost, llen, mask, orep, orsz, rmask, sid, rid)
    return src, lens, mask, rmask, sid, rid, orep, orsz, lost, llen, oout, olen, ost


@pytest.mark.parametrize("G,chunk,depth,explicit_ids",
                         [(37, 8, 3, True), (16, 16, 2, True), (5, 2, 4, True),
                          (37, 8, 3, False), (9, 4, 2, False)])
def test_pipeline_matches_oracle(gpu, G, chunk, depth, explicit_ids):
    """Every chunk (chunk < G included) reproduces the oracle over the whole batch: payloads,
    decoded sizes, repair symbol lengths and status -- with explicit id bases and with the
    defaults (g*k / g*r over the whole batch, not per chunk)."""
    import torch
    from netcode_amd import status_to_numpy
    from netcode_amd.pipeline import HostPipeline
    k, r, S = 24, 6, 2048
    src, lens, mask, rmask, sid, rid, orep, orsz, lost, llen, oout, olen, ost = \
        case(G, k, r, S, 7 + G, explicit_ids)
    if explicit_ids:
        d_sid = torch.from_numpy(sid.view(np.int32).copy()).to(gpu)
        d_rid = torch.from_numpy(rid.view(np.int32).copy()).to(gpu)
    else:
        d_sid = d_rid = None
    p = HostPipeline(k, r, S, chunk, gpu, depth)

    # encode alone
    h_rep = torch.empty((G, r, S), dtype=torch.uint8).pin_memory()
    h_rsz = torch.empty((G, r), dtype=torch.int16).pin_memory()
    h_rlen = torch.zeros((G,), dtype=torch.int16).pin_memory()
    p.encode(pinned(src), pinned(lens), h_rep, h_rsz, d_sid, d_rid, h_rep_len=h_rlen)
    torch.cuda.synchronize(gpu)
    assert (h_rep.numpy() == orep).all()
    assert (h_rsz.numpy().view(np.uint16) == orsz).all()
    assert (h_rlen.numpy().view(np.uint16) == lens.max(axis=1)).all()   # detail/encoder.cc:26,44-48

    # decode alone, repairs from the host
    h_rx, h_st = pinned(lost), torch.empty((G, 12), dtype=torch.uint8).pin_memory()
    h_rxlen = pinned(llen)
    p.decode(h_rx, h_rxlen, pinned(mask), h_rep, h_rsz, pinned(rmask), h_st, d_sid, d_rid)
    torch.cuda.synchronize(gpu)
    assert (status_to_numpy(h_st) == ost).all()
    assert (h_rx.numpy() == oout).all()
    assert (h_rxlen.numpy().view(np.uint16) == olen).all()

    # loopback encode_decode
    h_rep2 = torch.zeros((G, r, S), dtype=torch.uint8).pin_memory()
    h_rsz2 = torch.zeros((G, r), dtype=torch.int16).pin_memory()
    h_rx2, h_st2 = pinned(lost), torch.zeros((G, 12), dtype=torch.uint8).pin_memory()
    h_rxlen2 = pinned(llen)
    p.encode_decode(pinned(src), pinned(lens), h_rep2, h_rsz2, h_rx2, h_rxlen2, pinned(mask),
                    pinned(rmask), h_st2, d_sid, d_rid)
    torch.cuda.synchronize(gpu)
    assert (h_rep2.numpy() == orep).all()
    assert (status_to_numpy(h_st2) == ost).all()
    assert (h_rx2.numpy() == oout).all()
    assert (h_rxlen2.numpy().view(np.uint16) == olen).all()


def test_pipeline_rejects_bad_shapes(gpu):
    """Host tensors of the wrong dtype / trailing shape raise instead of being cast or broadcast
    by copy_."""
    import torch
    from netcode_amd.pipeline import HostPipeline
    p = HostPipeline(4, 2, 64, 2, gpu, 2)
    ok = dict(h_src=torch.zeros((3, 4, 64), dtype=torch.uint8).pin_memory(),
              h_src_len=torch.zeros((3, 4), dtype=torch.int16).pin_memory(),
              h_rep=torch.zeros((3, 2, 64), dtype=torch.uint8).pin_memory(),
              h_rep_size=torch.zeros((3, 2), dtype=torch.int16).pin_memory())
    p.encode(**ok)
    torch.cuda.synchronize(gpu)
    for name, bad in (("h_src_len", torch.zeros((3, 4), dtype=torch.int32).pin_memory()),
                      ("h_src", torch.zeros((3, 4, 32), dtype=torch.uint8).pin_memory()),
                      ("h_rep_size", torch.zeros((3, 1), dtype=torch.int16).pin_memory())):
        args = dict(ok)
        args[name] = bad
        with pytest.raises((ValueError, TypeError)):
            p.encode(**args)


def test_pipeline_rejects_pageable(gpu):
    import torch
    from netcode_amd.pipeline import HostPipeline
    p = HostPipeline(4, 2, 64, 2, gpu, 2)
    src = torch.zeros((3, 4, 64), dtype=torch.uint8)          # not pinned
    with pytest.raises(ValueError):
        p.encode(src, torch.zeros((3, 4), dtype=torch.int16).pin_memory(),
                 torch.zeros((3, 2, 64), dtype=torch.uint8).pin_memory(),
                 torch.zeros((3, 2), dtype=torch.int16).pin_memory())
