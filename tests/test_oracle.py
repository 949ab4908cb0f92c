"""CPU tests: the oracle against the reference's pinned behaviour (runs without a GPU).

Mirrors the reference's own tests where they pin results:
  tests/netcode/detail/test_galois_field.cc:15-26   (x * 1/x == 1)
  tests/netcode/detail/test_invert_matrix.cc:123-233 (jerasure equality, singular 3x3, M*M^-1=I)
  tests/netcode/test_reconstruction.cc:21-120        (encode one source / two sizes round trips)
  tests/end_to_end.cc                               (golden counters)
plus SURVEY §8(c) wire-format / coefficient KATs (tests/golden/kat.json).
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "kat.json")))


def test_field_inverse_all(oracle):
    for x in range(1, 256):
        assert oracle.gf_mul(x, oracle.gf_inv(x)) == 1


def test_kat_scalars(oracle):
    for rid, sid, c in KAT["coefficients"]:
        assert oracle.coefficient(rid, sid) == c
    for x, inv in KAT["inverses"]:
        assert oracle.gf_inv(x) == inv
    for a, b, p in KAT["products"]:
        assert oracle.gf_mul(a, b) == p
    for size, c, out in KAT["multiply_size"]:
        assert oracle.multiply_size(size, c) == out


def test_coefficient_uint32_wraparound(oracle):
    # galois_field.hh:156 computes in uint32: the product wraps before % 255.
    for rid, sid in [(0xFFFFFFFF, 5), (2_000_000, 8_000_000), (65535 * 32 + 31, 65535 * 128 + 127),
                     (123456789, 987654321)]:
        R = (rid + 1) & 0xFFFFFFFF
        S = (sid + 1) & 0xFFFFFFFF
        expect = (((R + S) & 0xFFFFFFFF) * R & 0xFFFFFFFF) % 255 + 1
        assert oracle.coefficient(rid, sid) == expect


def test_wire_kat(oracle):
    k = KAT["wire_rate2_abcd_efghij"]
    enc = oracle.Encoder()
    enc.set_rate(k["inputs"]["rate"])
    for d in k["inputs"]["data"]:
        enc.add_data(bytes.fromhex(d))
    assert [p.hex() for p in enc.packets] == k["packets"]


@pytest.mark.parametrize("n", ["1000", "10000"])
def test_end_to_end_golden(oracle, n):
    rc, got = oracle.end_to_end(int(n))
    assert rc == 0
    assert got == KAT["end_to_end"][n]


def test_invert_matches_jerasure_and_identity(oracle):
    mul = oracle.mul_table()
    m = np.array(KAT["invert_3x3_0_to_8_invertible"]["colmajor_input"], np.uint32)
    fail, inv = oracle.invert(m)
    assert fail is None
    M = m.reshape(3, 3).T      # logical M(i, j) = storage[j*3+i]
    I = inv.reshape(3, 3).T
    prod = np.zeros((3, 3), np.uint32)
    for i in range(3):
        for j in range(3):
            acc = 0
            for t in range(3):
                acc ^= int(mul[M[i, t], I[t, j]])
            prod[i, j] = acc
    assert (prod == np.eye(3, dtype=np.uint32)).all()


def test_invert_singular_reports_last_index(oracle):
    m = np.zeros(9, np.uint32)
    k = 0
    for i in range(3):
        for j in range(3):
            m[k] = (k + i) * 2
            k += 1
    fail, _ = oracle.invert(m)
    assert fail == KAT["invert_3x3_singular"]["expected_failure_index"]


def test_reconstruct_one_source(oracle):
    # test_reconstruction.cc "Encode one source"
    src = np.zeros((1, 1, 16), np.uint8)
    src[0, 0, :4] = np.frombuffer(b"abcd", np.uint8)
    rep, rsz = oracle.encode_batch(src, np.array([[4]], np.uint16), 1, 1,
                                   np.array([0], np.uint32), np.array([0], np.uint32))
    inv = oracle.gf_inv(oracle.coefficient(0, 0))
    assert oracle.multiply_size(int(rsz[0, 0]), inv) == 4
    mul = oracle.mul_table()
    assert bytes(mul[inv][rep[0, 0, :4]]) == b"abcd"


def test_simd_region_matches_scalar(oracle):
    rng = np.random.default_rng(0)
    L = oracle.lib()
    for n in [0, 1, 31, 32, 33, 1000, 4096]:
        src = rng.integers(0, 256, n + 1, dtype=np.uint8)
        for c in [0, 1, 2, 0x53, 255]:
            d0 = rng.integers(0, 256, n + 1, dtype=np.uint8)
            d1 = d0.copy()
            L.or_region_muladd(oracle._p(src), oracle._p(d0), n, c)
            L.or_region_muladd_simd(oracle._p(src), oracle._p(d1), n, c)
            assert (d0 == d1).all()


def test_gfni_region_matches_scalar(oracle):
    """The GFNI affine-matrix region MAC (the CPU upper-bound leg; or_set_simd(2)) gives the
    scalar 0x11D products for every coefficient."""
    L = oracle.lib()
    if not L.or_have_gfni():
        pytest.skip("no GFNI / AVX-512BW on this CPU")
    rng = np.random.default_rng(1)
    L.or_set_simd(2)
    try:
        for n in [0, 1, 63, 64, 65, 1000, 4096]:
            src = rng.integers(0, 256, n + 1, dtype=np.uint8)
            for c in range(256):
                d0 = rng.integers(0, 256, n + 1, dtype=np.uint8)
                d1 = d0.copy()
                L.or_set_simd(0)
                L.or_region_muladd(oracle._p(src), oracle._p(d0), n, c)
                L.or_set_simd(2)
                L.or_region_muladd(oracle._p(src), oracle._p(d1), n, c)
                assert (d0 == d1).all(), (n, c)
    finally:
        L.or_set_simd(0)


def test_generation_decode_round_trip_and_states(oracle):
    from helpers import loss_exact_m, make_sources
    G, k, r, S = 20, 32, 8, 256
    src, lens = make_sources(G, k, S, S, seed=3, ragged=True)
    rep, rsz = oracle.encode_batch(src, lens, k, r)
    mask = loss_exact_m(G, k, 8, seed=4)
    lost = src.copy()
    lost[mask == 0] = 0
    llen = lens.copy()
    llen[mask == 0] = 0
    out, olen, st = oracle.decode_batch(lost, llen, mask, rep, rsz, np.ones((G, r), np.uint8))
    for g in range(G):
        if st["state"][g] == 0:
            assert (out[g] == src[g]).all() and (olen[g] == lens[g]).all()
            assert st["nb_decoded"][g] == 8
        else:
            assert st["state"][g] == 3
    assert (st["state"] == 0).sum() >= G - 3


def test_streaming_decoder_recovers_lost_source(oracle):
    # tests/netcode/test_decoder.cc "Decoder repairs a lost source" shape: rate 2, lose source 0.
    enc = oracle.Encoder()
    enc.set_rate(2)
    enc.add_data(b"abcd")
    enc.add_data(b"efghij")
    dec = oracle.Decoder(in_order=False)
    dec.add_packet(enc.packets[1])   # source 1
    dec.add_packet(enc.packets[2])   # repair 0 covering {0,1}
    assert sorted(dec.data) == [(0, b"abcd"), (1, b"efghij")]
    assert dec.nb_decoded == 1


def test_golden_fixtures_reproduce(oracle):
    """The committed decode fixtures are reproduced by the current oracle (regression pin)."""
    for name in ["gen_k16_r4_loss25", "gen_k32_r8_ragged"]:
        z = np.load(os.path.join(HERE, "golden", name + ".npz"))
        k, r = z["src"].shape[1], z["rep"].shape[1]
        rep, rsz = oracle.encode_batch(z["src"], z["src_len"], k, r, z["sid_base"], z["rid_base"])
        assert (rep == z["rep"]).all() and (rsz == z["rep_size"]).all()
        lost = z["src"].copy()
        lost[z["src_mask"] == 0] = 0
        llen = z["src_len"].copy()
        llen[z["src_mask"] == 0] = 0
        out, olen, st = oracle.decode_batch(lost, llen, z["src_mask"], rep, rsz, z["rep_mask"],
                                            z["sid_base"], z["rid_base"])
        assert (out == z["out"]).all() and (olen == z["out_len"]).all()
        assert (st.view(np.uint8).reshape(len(st), -1) == z["status"]).all()


def test_dense_oracle_round_trip_and_inverse(oracle):
    """Dense extension (config 5): or_dense_decode inverts with the reference's own invert
    (invert_matrix.cc:9-128) -- M * M^-1 = I, decode(encode(x)) = x, singular reported."""
    rng = np.random.default_rng(11)
    T = oracle.mul_table()
    for n in (1, 7, 48):
        mat = rng.integers(0, 256, (n, n), dtype=np.uint8)
        src = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        ok, out, inv = oracle.dense_decode(mat, oracle.dense_encode(mat, src))
        if not ok:
            continue
        assert (out == src).all()
        prod = np.zeros((n, n), np.uint8)
        for i in range(n):
            for j in range(n):
                acc = 0
                for t in range(n):
                    acc ^= int(T[mat[i, t], inv[t, j]])
                prod[i, j] = acc
        assert (prod == np.eye(n, dtype=np.uint8)).all()
    mat = rng.integers(0, 256, (8, 8), dtype=np.uint8)
    mat[3] = mat[1]
    ok, out, inv = oracle.dense_decode(mat, np.zeros((8, 16), np.uint8))
    assert not ok and not out.any() and not inv.any()
