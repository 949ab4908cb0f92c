"""GPU parity of the device wire format (ntc_gf256_write_repairs / write_sources / read_packets,
include/netcode/gpu.h) against the oracle's packetizer restatement, byte for byte, and an
end-to-end encode -> serialise -> lose -> parse -> decode round trip on the device."""
import numpy as np
import pytest

from helpers import loss_iid, make_sources
from wire_cases import batch_packets, ids_rle_by_hand, repair_packet_by_hand, to_slots

pytestmark = pytest.mark.gpu


def dev(a, d):
    import torch
    a = np.ascontiguousarray(a)
    view = {np.dtype(np.uint16): np.int16, np.dtype(np.uint32): np.int32}.get(a.dtype)
    return torch.from_numpy((a.view(view) if view else a).copy()).to(d)


def ids_of(mode, G, k, r):
    if mode == "default":
        return None, None, np.arange(G, dtype=np.uint64) * k, np.arange(G, dtype=np.uint64) * r
    if mode == "wrap":    # config 4: ids of a 65536-generation run
        base = 65536 - G
        s = ((base + np.arange(G, dtype=np.uint64)) * k).astype(np.uint32)
        q = ((base + np.arange(G, dtype=np.uint64)) * r).astype(np.uint32)
    else:
        s = (np.arange(G, dtype=np.uint64) * k + 11).astype(np.uint32)
        q = (np.arange(G, dtype=np.uint64) * r + 5).astype(np.uint32)
    return s, q, s.astype(np.uint64), q.astype(np.uint64)


SHAPES = [
    # G, k, r, S, stride, ragged, ids
    (16, 32, 8, 1024, 1024, False, "default"),
    (6, 128, 32, 4096, 4096, False, "offset"),
    (8, 128, 32, 1500, 1504, True, "wrap"),
    (4, 300, 3, 100, 112, True, "offset"),      # id list of 2 runs
    (3, 1, 1, 16, 16, True, "default"),         # k = 1: id list without runs
    (5, 9, 12, 2080, 2080, True, "offset"),
]


@pytest.mark.parametrize("G,k,r,S,stride,ragged,ids", SHAPES)
def test_write_repairs_and_sources_parity(gpu, oracle, G, k, r, S, stride, ragged, ids):
    import torch
    from netcode_amd import BatchEncoder, Wire
    src, lens = make_sources(G, k, S, stride, seed=3 * G + k, ragged=ragged)
    sid, rid, sidv, ridv = ids_of(ids, G, k, r)
    s_t, l_t = dev(src, gpu), dev(lens, gpu)
    sid_t = None if sid is None else dev(sid, gpu)
    rid_t = None if rid is None else dev(rid, gpu)
    enc = BatchEncoder(k, r, gpu)(s_t, l_t, sid_t, rid_t)
    w = Wire(gpu)
    rp, rl = w.write_repairs(enc, k, sid_t, rid_t)
    sp, sl = w.write_sources(s_t, l_t, sid_t)
    torch.cuda.synchronize()
    rep = enc.repairs.cpu().numpy()
    esz = enc.encoded_size.cpu().numpy().view(np.uint16)
    symlen = enc.symbol_len.cpu().numpy().view(np.uint16)
    rp, rl, sp, sl = rp.cpu().numpy(), rl.cpu().numpy(), sp.cpu().numpy(), sl.cpu().numpy()
    for g in range(G):
        ids_g = (sidv[g] + np.arange(k, dtype=np.uint64)) & 0xFFFFFFFF
        for j in range(r):
            want = oracle.write_repair_packet(int(ridv[g]) + j, rep[g, j, :symlen[g]], ids_g,
                                              int(esz[g, j]))
            p = g * r + j
            assert rl[p] == len(want), (g, j)
            assert rp[p, :rl[p]].tobytes() == want, (g, j)
        for i in range(k):
            want = oracle.write_source_packet(int(sidv[g]) + i, src[g, i, :lens[g, i]])
            p = g * k + i
            assert sl[p] == len(want) and sp[p, :sl[p]].tobytes() == want, (g, i)


@pytest.mark.parametrize("G,k,r,S,stride,sid0,rid0", [
    (6, 16, 4, 1024, 1024, 0, 0),
    (5, 33, 7, 100, 112, 11, 5),
    (4, 300, 3, 64, 64, 0xFFFF0000, 17),
    (3, 128, 32, 4096, 4096, 128 * 1000, 32 * 1000),
])
def test_read_packets_parity(gpu, oracle, G, k, r, S, stride, sid0, rid0):
    import torch
    from netcode_amd import Wire
    pk, src, lens = batch_packets(oracle, G, k, r, S, stride, sid0, rid0, seed=5 * G + r)
    sym = np.arange(16, dtype=np.uint8)
    sidb = sid0
    # hand-encoded id lists for repairs rid0+1 / rid0+2 (replacing any regular packet of those ids)
    taken = {(rid0 + 1) & 0xFFFFFFFF, (rid0 + 2) & 0xFFFFFFFF}
    pk = [p for p in pk if not (len(p) >= 5 and p[0] == 1 and int.from_bytes(p[1:5], "big") in taken)]
    pk += [repair_packet_by_hand(rid0 + 1, sym, ids_rle_by_hand(sidb, [(5, 1), (3, 0), (k - 6, 1)]), 3)
           if k > 6 else b"",
           repair_packet_by_hand(rid0 + 2, sym, ids_rle_by_hand(sidb, [(k - 2, 1)]), 3)]
    buf, plen = to_slots(pk)
    rb = Wire(gpu).read_packets(dev(buf, gpu), dev(plen, gpu), G, k, r, stride, sid0, rid0)
    torch.cuda.synchronize()
    s, sl, sm, rep, rsz, rm, st = oracle.read_packets(pk, G, k, r, stride, sid0, rid0)
    assert (rb.status.cpu().numpy() == st).all()
    gsm, grm = rb.src_mask.cpu().numpy(), rb.rep_mask.cpu().numpy()
    assert (gsm == sm).all() and (grm == rm).all()
    assert (rb.src_len.cpu().numpy().view(np.uint16) == sl).all()
    assert (rb.rep_size.cpu().numpy().view(np.uint16) == rsz).all()
    gs, gr = rb.src.cpu().numpy(), rb.rep.cpu().numpy()
    assert (gs[sm == 1] == s[sm == 1]).all()
    assert (gr[rm == 1] == rep[rm == 1]).all()


def test_wire_round_trip_decode(gpu, oracle):
    """Config-3 shape: encode, serialise sources + repairs on the device, drop ~12 % of the
    packets, parse the survivors on the device, decode; decoded generations reproduce their
    sources and every status equals the oracle's decode of the same losses."""
    import torch
    from netcode_amd import BatchDecoder, BatchEncoder, Wire, status_to_numpy
    G, k, r, S = 32, 128, 32, 4096
    src, lens = make_sources(G, k, S, S, seed=77, ragged=True)
    s_t, l_t = dev(src, gpu), dev(lens, gpu)
    enc = BatchEncoder(k, r, gpu)(s_t, l_t)
    w = Wire(gpu)
    sp, sl = w.write_sources(s_t, l_t)
    rp, rl = w.write_repairs(enc, k)
    keep_s = loss_iid((G * k,), 0.12, 5).astype(bool)
    keep_r = loss_iid((G * r,), 0.12, 6).astype(bool)
    stride_p = max(sp.shape[1], rp.shape[1])
    pk = torch.zeros((int(keep_s.sum() + keep_r.sum()), stride_p), dtype=torch.uint8, device=gpu)
    ks = torch.from_numpy(np.nonzero(keep_s)[0]).to(gpu)
    kr = torch.from_numpy(np.nonzero(keep_r)[0]).to(gpu)
    ns = len(ks)
    pk[:ns, :sp.shape[1]] = sp[ks]
    pk[ns:, :rp.shape[1]] = rp[kr]
    plen = torch.cat([sl[ks], rl[kr]])
    perm = torch.randperm(len(plen), device=gpu, generator=torch.Generator(device=gpu).manual_seed(1))
    rb = w.read_packets(pk[perm].contiguous(), plen[perm].contiguous(), G, k, r, S)
    st = BatchDecoder(k, r, gpu)(rb.src, rb.src_len, rb.src_mask, rb.rep, rb.rep_size, rb.rep_mask)
    torch.cuda.synchronize()
    assert (rb.status.cpu().numpy() <= 1).all()
    smask = keep_s.reshape(G, k).astype(np.uint8)
    rmask = keep_r.reshape(G, r).astype(np.uint8)
    assert (rb.src_mask.cpu().numpy() == smask).all() and (rb.rep_mask.cpu().numpy() == rmask).all()
    gst = status_to_numpy(st)
    orep, orsz = oracle.encode_batch(src, lens, k, r)
    lost = src * smask[:, :, None]
    _, _, ost = oracle.decode_batch(lost, lens * smask, smask, orep, orsz, rmask)
    assert (gst == ost).all()
    ok = gst["state"] <= 1
    assert ok.any()
    assert (rb.src.cpu().numpy()[ok] == src[ok]).all()
    assert (rb.src_len.cpu().numpy().view(np.uint16)[ok] == lens[ok]).all()
