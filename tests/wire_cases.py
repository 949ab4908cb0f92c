"""Wire-format test material shared by the CPU and GPU wire tests: packet lists built with the
oracle's packetizer restatement (oracle/ntc_oracle.c, packetizer.hh:90-122, 165-183), including
the malformed packets whose statuses ntc_gf256_read_packets must reproduce."""
import struct

import numpy as np

from helpers import make_sources


def batch_packets(oracle, G, k, r, S, stride, sid0, rid0, seed, p_src=0.7, p_rep=0.8, ragged=True):
    """Encode a batch with the oracle and serialise a random subset of its sources and repairs,
    plus one packet of every malformed kind; returns (packets, src, src_len)."""
    rng = np.random.default_rng(seed)
    src, lens = make_sources(G, k, S, stride, seed=seed, ragged=ragged)
    sid = (sid0 + np.arange(G, dtype=np.uint64) * k).astype(np.uint32)
    rid = (rid0 + np.arange(G, dtype=np.uint64) * r).astype(np.uint32)
    rep, rsz = oracle.encode_batch(src, lens, k, r, sid, rid)
    pk = []
    for g in range(G):
        for i in range(k):
            if rng.random() < p_src:
                pk.append(oracle.write_source_packet(int(sid[g]) + i, src[g, i, :lens[g, i]]))
        symsz = int(lens[g].max())
        ids = int(sid[g]) + np.arange(k, dtype=np.uint64)
        for j in range(r):
            if rng.random() < p_rep:
                pk.append(oracle.write_repair_packet(int(rid[g]) + j, rep[g, j, :symsz], ids,
                                                     int(rsz[g, j])))
    # malformed and foreign packets (statuses NTC_PKT_*)
    good_src = oracle.write_source_packet(int(sid[0]), src[0, 0, :lens[0, 0]])
    ids0 = int(sid[0]) + np.arange(k, dtype=np.uint64)
    good_rep = oracle.write_repair_packet(int(rid[0]), rep[0, 0, :int(lens[0].max())], ids0,
                                          int(rsz[0, 0]))
    junk = [
        b"",                                                    # empty -> overflow
        bytes([0, 0, 3, 0, 0]),                                 # ack
        bytes([9, 1, 2, 3]),                                    # unknown type
        good_src[:5],                                           # truncated header
        good_src[:-1] if len(good_src) > 7 else good_src[:6],   # truncated payload
        good_rep[:7 + int(lens[0].max()) + 3],                  # truncated id list
        oracle.write_source_packet((int(sid0) + G * k + 5) & 0xFFFFFFFF, src[0, 0, :4]),  # out
        oracle.write_repair_packet((int(rid0) - 1) & 0xFFFFFFFF, rep[0, 0, :8], ids0, 1),  # out
        oracle.write_source_packet(int(sid[0]) + 1, np.zeros(stride + 16, np.uint8)),      # large
        oracle.write_repair_packet(int(rid[0]) + 1, rep[0, 1, :8], ids0[1:], 7),  # not the gen.
        oracle.write_repair_packet(int(rid[0]) + 1, rep[0, 1, :8],
                                   np.concatenate([ids0[:-1], ids0[-1:] + 1]), 7),  # gap
    ]
    pk = pk + junk
    order = rng.permutation(len(pk))
    return [pk[i] for i in order], src, lens


def ids_rle_by_hand(first, runs):
    """A run-length id list written by hand (count, first, (run, delta)...) -- lets tests feed
    encodings the oracle's writer never produces (runs of delta 0, short runs)."""
    split = []
    for run, delta in runs:                   # runs longer than 255 continue in the next entry
        while run > 255:
            split.append((255, delta))
            run -= 255
        split.append((run, delta))
    b = struct.pack(">HI", 1 + len(split), first)
    for run, delta in split:
        b += struct.pack(">BH", run, delta)
    return b


def repair_packet_by_hand(rid, sym, ids_blob, esz):
    sym = bytes(sym)
    return (struct.pack(">BIH", 1, rid, len(sym)) + sym + ids_blob + struct.pack(">HH", esz, len(sym))
            + sym)


def to_slots(packets, pkt_stride=None):
    n = len(packets)
    mx = max([len(p) for p in packets] + [1])
    pkt_stride = pkt_stride or (mx + 15) // 16 * 16
    buf = np.zeros((n, pkt_stride), np.uint8)
    lens = np.zeros(n, np.uint32)
    for i, p in enumerate(packets):
        buf[i, :len(p)] = np.frombuffer(p, np.uint8)
        lens[i] = len(p)
    return buf, lens
