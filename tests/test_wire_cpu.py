"""CPU tests of the wire-format specification (oracle restatement of netcode/detail/packetizer.hh)
and of the host-side sizing helper of the device wire ABI (include/netcode/gpu.h)."""
import numpy as np
import pytest

from wire_cases import batch_packets, ids_rle_by_hand, repair_packet_by_hand


def test_oracle_wire_kat(oracle):
    """SURVEY §8(c) known-answer packets (hand-verified: c(0,0)=3, c(0,1)=4 over 0x11D)."""
    rep = oracle.write_repair_packet(0, np.frombuffer(bytes.fromhex("2a232411b9b5"), np.uint8),
                                     [0, 1], 0x14)
    assert rep.hex() == "01" "00000000" "0006" "2a232411b9b5" "0002" "00000000" "01" "0001" \
        "0014" "0006" "2a232411b9b5"
    assert oracle.write_source_packet(0, np.frombuffer(b"abcd", np.uint8)).hex() == \
        "02" "00000000" "0004" "61626364"
    assert oracle.write_source_packet(1, np.frombuffer(b"efghij", np.uint8)).hex() == \
        "02" "00000001" "0006" "65666768696a"


def test_oracle_id_list_runs(oracle):
    """write_ids groups equal deltas in runs of at most 255 (packetizer.hh:263-309)."""
    k = 600
    p = oracle.write_repair_packet(7, np.zeros(4, np.uint8), np.arange(100, 100 + k), 0)
    ids = p[7 + 4:]
    count = int.from_bytes(ids[:2], "big")
    assert count == 1 + 3                      # 599 deltas of 1 -> runs 255, 255, 89
    assert int.from_bytes(ids[2:6], "big") == 100
    runs = [(ids[6 + 3 * i], int.from_bytes(ids[7 + 3 * i:9 + 3 * i], "big")) for i in range(3)]
    assert runs == [(255, 1), (255, 1), (89, 1)]


@pytest.mark.parametrize("G,k,r,S,stride,sid0,rid0", [
    (6, 16, 4, 1024, 1024, 0, 0),
    (5, 33, 7, 100, 112, 11, 5),
    (4, 300, 3, 64, 64, 0xFFFF0000, 17),      # 2 id runs; ids near the top of the u32 range
])
def test_oracle_read_packets_round_trip(oracle, G, k, r, S, stride, sid0, rid0):
    pk, src, lens = batch_packets(oracle, G, k, r, S, stride, sid0, rid0, seed=G + k)
    s, sl, sm, rep, rsz, rm, st = oracle.read_packets(pk, G, k, r, stride, sid0, rid0)
    # junk statuses: empty, ack, bad type, 2 truncations, truncated ids, 2 out, large, 2 not-gen
    counts = np.bincount(st, minlength=8)
    assert counts[2] == 1 and counts[3] == 1 and counts[4] == 4 and counts[5] == 2
    assert counts[6] == 1 and counts[7] == 2
    got = sm.astype(bool)
    assert (s[got] == src[got]).all() and (sl[got] == lens[got]).all()
    assert (s[~got] == 0).all()
    # the batch decodes from what was received, exactly as from the generation layout directly
    sid = (sid0 + np.arange(G, dtype=np.uint64) * k).astype(np.uint32)
    rid = (rid0 + np.arange(G, dtype=np.uint64) * r).astype(np.uint32)
    out, olen, ost = oracle.decode_batch(s, sl, sm, rep, rsz, rm, sid, rid)
    ok = ost["state"] <= 1
    assert (out[ok] == src[ok]).all() and (olen[ok] == lens[ok]).all()


def test_oracle_read_accepts_equivalent_id_encodings(oracle):
    """read_ids builds a set: any run-length encoding of the generation's ids is the same repair
    (split runs, runs of delta 0 that only repeat an id)."""
    k, stride = 20, 32
    sym = np.arange(16, dtype=np.uint8)
    cases = {
        ids_rle_by_hand(0, [(19, 1)]): 1,
        ids_rle_by_hand(0, [(5, 1), (14, 1)]): 1,
        ids_rle_by_hand(0, [(5, 1), (3, 0), (14, 1)]): 1,
        ids_rle_by_hand(0, [(0, 7), (19, 1)]): 1,            # an empty run is ignored
        ids_rle_by_hand(0, [(18, 1)]): 7,                    # one id short
        ids_rle_by_hand(1, [(19, 1)]): 7,                    # shifted
        ids_rle_by_hand(0, [(10, 1), (1, 2), (8, 1)]): 7,    # gap
    }
    for blob, want in cases.items():
        p = repair_packet_by_hand(0, sym, blob, 3)
        st = oracle.read_packets([p], 1, k, 2, stride)[-1]
        assert st[0] == want, (blob.hex(), st[0])


def test_repair_packet_bytes_helper(native_built):
    from netcode_amd import _native
    L = _native.load()
    for k, stride in [(1, 16), (2, 16), (128, 4096), (256, 1504), (1000, 65536)]:
        ids = 6 + 3 * ((k - 1 + 254) // 255)
        want = (11 + 2 * stride + ids + 15) // 16 * 16
        assert L.ntc_gf256_repair_packet_bytes(k, stride) == want
