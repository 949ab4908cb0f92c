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

    # loopback moving only received rows in and lost rows out (packed)
    h_mask = pinned(mask)
    _, _, n_rx, n_lost = HostPipeline.row_bases(h_mask)
    assert n_rx == int(mask.sum()) and n_lost == mask.size - n_rx
    h_rxp = pinned(src[mask != 0])
    h_rec = torch.full((n_lost, S), 0xAB, dtype=torch.uint8).pin_memory()
    h_rep3 = torch.zeros((G, r, S), dtype=torch.uint8).pin_memory()
    h_rsz3 = torch.zeros((G, r), dtype=torch.int16).pin_memory()
    h_st3 = torch.zeros((G, 12), dtype=torch.uint8).pin_memory()
    h_rxlen3 = pinned(llen)
    p.encode_decode_packed(pinned(src), pinned(lens), h_rep3, h_rsz3, h_rxp, h_rxlen3, h_mask,
                           pinned(rmask), h_rec, h_st3, d_sid, d_rid)
    torch.cuda.synchronize(gpu)
    assert (h_rep3.numpy() == orep).all()
    assert (status_to_numpy(h_st3) == ost).all()
    assert (h_rxlen3.numpy().view(np.uint16) == olen).all()
    # lost slots, packed in (generation, slot) order: the oracle's recovered bytes (zeros where
    # the oracle left the slot untouched, i.e. the zeroed lost slot)
    assert (h_rec.numpy() == oout[mask == 0]).all()


@pytest.mark.parametrize("k,stride,want,zero_rest", [(24, 64, 1, True), (300, 32, 0, False),
                                                     (7, 4096, 1, False)])
def test_pack_unpack_slots(gpu, k, stride, want, zero_rest):
    """ntc_gf256_unpack_slots / ntc_gf256_pack_slots against numpy boolean indexing, with a
    chunk-relative packed buffer (row0) and generations with no selected slot."""
    import torch
    from netcode_amd import Wire
    rng = np.random.default_rng(k + stride)
    G = 11
    mask = (rng.random((G, k)) < 0.6).astype(np.uint8) * rng.integers(1, 256, (G, k), dtype=np.uint8)
    mask[3] = 0
    mask[5] = 1
    sel = (mask != 0) == bool(want)
    cnt = sel.sum(1)
    base = np.cumsum(cnt) - cnt + 5                      # rows numbered from row0 = 5
    n = int(cnt.sum())
    packed = rng.integers(0, 256, (max(n, 1), stride), dtype=np.uint8)
    slots0 = rng.integers(0, 256, (G, k, stride), dtype=np.uint8)
    w = Wire(gpu)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(gpu)
    d_slots = d(slots0)
    d_mask, d_base = d(mask), d(base.astype(np.int32))
    w.unpack_slots(d(packed), d_base, d_mask, d_slots, want=want, zero_rest=zero_rest, row0=5)
    exp = slots0.copy()
    exp[sel] = packed[:n]
    if zero_rest:
        exp[~sel] = 0
    assert (d_slots.cpu().numpy() == exp).all()
    out = d(np.zeros((max(n, 1), stride), np.uint8))
    w.pack_slots(d(slots0), d_mask, d_base, out, want=want, row0=5)
    assert (out.cpu().numpy()[:n] == slots0[sel]).all()


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


@pytest.mark.parametrize("G,chunk,depth,S", [(21, 8, 3, 1024), (6, 6, 2, 1500)])
def test_wire_pipeline_matches_oracle(gpu, G, chunk, depth, S):
    """HostPipeline.encode_decode_wire (socket buffer to socket buffer in the reference's wire
    format): the sender's repair packets equal the oracle's packetizer (packetizer.hh:90-122) over
    the oracle's repairs; the receiver, fed the received source packets (oracle packetizer,
    packetizer.hh:165-183) and the sender's repair packets, returns the oracle's status, recovered
    rows and decoded sizes.  Continuous ids that wrap u32 between generations."""
    import torch
    from netcode_amd import Wire, status_to_numpy
    from netcode_amd.pipeline import HostPipeline
    k, r = 16, 6
    stride = (S + 15) // 16 * 16
    src, lens = make_sources(G, k, S, stride, seed=G + S, ragged=True)
    mask = loss_mixed_m(G, k, r, seed=G + S + 1)
    g = np.arange(G, dtype=np.uint64)
    sid = ((2**32 - 3 * k + g * k) & 0xFFFFFFFF).astype(np.uint32)
    rid = ((2**32 - 2 * r + g * r) & 0xFFFFFFFF).astype(np.uint32)
    orep, orsz = O.encode_batch(src, lens, k, r, sid, rid)
    lost = src.copy()
    lost[mask == 0] = 0
    llen = lens * (mask != 0)
    oout, olen, ost = O.decode_batch(lost, llen, mask, orep, orsz, np.ones((G, r), np.uint8), sid, rid)
    sps = Wire.source_packet_bytes(stride)
    pk, pl, first = [], [], [0]
    for gi in range(G):
        for i in range(k):
            if mask[gi, i]:
                p = O.write_source_packet(int(sid[gi]) + i, src[gi, i, :lens[gi, i]])
                pk.append(np.frombuffer(p.ljust(sps, b"\0"), np.uint8))
                pl.append(len(p))
        first.append(len(pk))
    h_rxp = torch.from_numpy(np.stack(pk)).pin_memory()
    h_rxl = torch.tensor(pl, dtype=torch.int32).pin_memory()
    rps = Wire.repair_packet_bytes(k, stride)
    h_rep_pkts = torch.zeros((G * r, rps), dtype=torch.uint8).pin_memory()
    h_rep_len = torch.zeros((G * r,), dtype=torch.int32).pin_memory()
    n_lost = int((mask == 0).sum())
    h_rec = torch.full((max(n_lost, 1), stride), 0xAB, dtype=torch.uint8).pin_memory()
    h_dec_len = torch.zeros((G, k), dtype=torch.int16).pin_memory()
    h_st = torch.zeros((G, 12), dtype=torch.uint8).pin_memory()
    d_sid = torch.from_numpy(sid.view(np.int32).copy()).to(gpu)
    d_rid = torch.from_numpy(rid.view(np.int32).copy()).to(gpu)
    p = HostPipeline(k, r, stride, chunk, gpu, depth)
    p.encode_decode_wire(pinned(src), pinned(lens), h_rep_pkts, h_rep_len, h_rxp, h_rxl,
                         torch.tensor(first), pinned(mask), h_rec[:n_lost], h_dec_len, h_st, sid, rid,
                         d_sid, d_rid)
    torch.cuda.synchronize(gpu)
    ids = lambda gi: (sid[gi].astype(np.uint64) + np.arange(k, dtype=np.uint64)) & 0xFFFFFFFF
    for gi in range(G):
        L = int(lens[gi].max())
        for j in range(r):
            ref = O.write_repair_packet(int(rid[gi]) + j, orep[gi, j, :L], ids(gi), int(orsz[gi, j]))
            n = int(h_rep_len[gi * r + j])
            assert h_rep_pkts[gi * r + j, :n].numpy().tobytes() == ref, (gi, j)
    st = status_to_numpy(h_st)
    assert (st == ost).all()
    dec = (ost["state"] == 0)
    lost_gen = np.nonzero(mask == 0)[0]
    sel = dec[lost_gen]
    assert (h_rec[:n_lost].numpy()[sel] == oout[mask == 0][sel]).all()
    assert (h_dec_len.numpy().view(np.uint16)[mask == 0][sel] == olen[mask == 0][sel]).all()


def test_wire_pipeline_rejects_non_contiguous_bases(gpu):
    """read_packets maps ids to slots from each chunk's first bases, so encode_decode_wire refuses
    id bases that are not contiguous within a chunk instead of misplacing packets."""
    import torch
    from netcode_amd import Wire
    from netcode_amd.pipeline import HostPipeline
    G, k, r, stride, chunk = 4, 8, 2, 64, 2
    src = torch.zeros((G, k, stride), dtype=torch.uint8).pin_memory()
    lens = torch.full((G, k), stride, dtype=torch.int16).pin_memory()
    mask = torch.ones((G, k), dtype=torch.uint8).pin_memory()
    rps, sps = Wire.repair_packet_bytes(k, stride), Wire.source_packet_bytes(stride)
    args = (src, lens, torch.zeros((G * r, rps), dtype=torch.uint8).pin_memory(),
            torch.zeros((G * r,), dtype=torch.int32).pin_memory(),
            torch.zeros((G * k, sps), dtype=torch.uint8).pin_memory(),
            torch.zeros((G * k,), dtype=torch.int32).pin_memory(),
            torch.arange(0, G * k + 1, k), mask, torch.zeros((1, stride), dtype=torch.uint8).pin_memory(),
            torch.zeros((G, k), dtype=torch.int16).pin_memory(),
            torch.zeros((G, 12), dtype=torch.uint8).pin_memory())
    sid = np.arange(G, dtype=np.uint32) * k
    rid = np.arange(G, dtype=np.uint32) * r
    sid[1] += 1                                     # generation 1 not at sid[0] + k
    d = lambda a: torch.from_numpy(a.view(np.int32).copy()).to(gpu)
    p = HostPipeline(k, r, stride, chunk, gpu, 2)
    with pytest.raises(ValueError, match="contiguous"):
        p.encode_decode_wire(*args, sid, rid, d(sid), d(rid))
