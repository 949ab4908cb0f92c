"""CPU tests of GF(2^w), w in {4, 8, 16, 32}: the oracle's restatement and the
library's host-side helpers (ntc_gf_*, include/netcode/gpu.h) against an independent pure-Python
carry-less reference, plus the field invariants the reference's own tests pin
(tests/netcode/test_galois_field.cc: x * x^-1 = 1).  For w != 8 the field bytes are "parity
unpinned" against the reference itself (gf-complete is absent); they follow gf-complete's published
default polynomials."""
import random

import numpy as np
import pytest

POLY = {4: 0x13, 8: 0x11D, 16: 0x1100B, 32: 0x100400007}
WS = (4, 8, 16, 32)


def py_mul(w, a, b):
    r = 0
    for i in range(w):
        if (b >> i) & 1:
            r ^= a << i
    for i in range(2 * w - 2, w - 1, -1):
        if (r >> i) & 1:
            r ^= POLY[w] << (i - w)
    return r


def py_coefficient(w, rid, sid):
    res = (((rid + 1) + (sid + 1)) * (rid + 1)) & 0xFFFFFFFF
    if w == 32:
        return res or 1
    return res % ((1 << w) - 1) + 1


def py_region(w, src: bytes, c: int) -> bytes:
    if w == 4:
        return bytes((py_mul(4, c, b >> 4) << 4) | py_mul(4, c, b & 15) for b in src)
    if w == 8:
        return bytes(py_mul(8, c, b) for b in src)
    wb = w // 8
    out = bytearray()
    for i in range(0, len(src), wb):
        x = int.from_bytes(src[i:i + wb], "little")
        out += py_mul(w, c, x).to_bytes(wb, "little")
    return bytes(out)


@pytest.mark.parametrize("w", WS)
def test_field_products_and_inverses(oracle, native_built, w):
    from netcode_amd import _native
    L = _native.load()
    rng = random.Random(w)
    for _ in range(300):
        a, b = rng.getrandbits(w), rng.getrandbits(w)
        want = py_mul(w, a, b)
        assert oracle.fw_mul(w, a, b) == want
        assert L.ntc_gf_multiply(w, a, b) == want
        if a:
            inv = L.ntc_gf_invert(w, a)
            assert py_mul(w, a, inv) == 1
            assert oracle.fw_inv(w, a) == inv
    # alpha^w reduces to the polynomial's low part
    assert py_mul(w, 1 << (w - 1), 2) == POLY[w] ^ (1 << w)


def test_known_products():
    assert py_mul(8, 0x53, 0xCA) == 0x8F            # SURVEY §8(c) KAT
    assert py_mul(4, 8, 2) == 0x3
    assert py_mul(16, 0x8000, 2) == 0x100B
    assert py_mul(32, 0x80000000, 2) == 0x400007


@pytest.mark.parametrize("w", WS)
def test_coefficient_and_size_coding(oracle, native_built, w):
    from netcode_amd import _native
    L = _native.load()
    rng = random.Random(100 + w)
    ids = [(0, 0), (1, 0), (3, 7), (31, 127), (0xFFFFFFFF, 1), (0xFFFF, 0xFFFFFFFF)]
    ids += [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(200)]
    for rid, sid in ids:
        c = py_coefficient(w, rid, sid)
        assert 1 <= c < (1 << w)
        assert L.ntc_gf_coefficient(w, rid, sid) == c == oracle.fw_coefficient(w, rid, sid)
    if w == 32:   # (rid+1) * ((rid+1)+(sid+1)) = 2^32 wraps to 0 -> 1 (galois_field.hh:147-153)
        assert L.ntc_gf_coefficient(32, 0xFFFF, 0xFFFFFFFF) == 1
    for size in (0, 1, 6, 1024, 1500, 4096, 65535):
        for c in (0, 1, 3, (1 << w) - 1, rng.getrandbits(w)):
            if w <= 8:
                want = int.from_bytes(py_region(w, size.to_bytes(2, "little"), c), "little") if c else 0
            else:
                want = py_mul(w, size, c) & 0xFFFF if size and c else 0   # w = 32 truncates
            assert L.ntc_gf_multiply_size(w, size, c) == want
            assert oracle.fw_multiply_size(w, size, c) == want


@pytest.mark.parametrize("w", WS)
def test_oracle_regions(oracle, w):
    rng = np.random.default_rng(w)
    for n in (4, 16, 1024, 1500):
        src = rng.integers(0, 256, n, dtype=np.uint8)
        dst = rng.integers(0, 256, n, dtype=np.uint8)
        c = int(rng.integers(1, 1 << min(w, 31)))
        want = np.frombuffer(py_region(w, src.tobytes(), c), np.uint8)
        assert (oracle.fw_region(w, src, dst, c, False) == want).all()
        assert (oracle.fw_region(w, src, dst, c, True) == (want ^ dst)).all()


@pytest.mark.parametrize("w", (4, 16, 32))
def test_oracle_stream_round_trip(oracle, w):
    """The oracle's streaming encoder/decoder restatement in GF(2^w): lossy in-order stream,
    every delivered datum equals what was sent (symbol sizes are whole field words)."""
    rng = np.random.default_rng(w)
    enc = oracle.Encoder(galois_field_size=w)
    enc.set_rate(3)
    enc.set_window_size(16)
    sent = []
    for i in range(200):
        d = rng.integers(0, 256, 4 * int(rng.integers(1, 200)), dtype=np.uint8).tobytes()
        sent.append(d)
        enc.add_data(d)
    dec = oracle.Decoder(in_order=True, galois_field_size=w)
    dec.set_ack_period_ms(0)
    for p in enc.packets:
        if rng.random() >= 0.15:
            dec.add_packet(p)
    assert dec.nb_decoded > 0
    if w != 32:     # w = 32 codes sizes with a truncated product (galois_field.hh:118)
        got = dict(dec.data)
        assert all(got[i] == sent[i] for i in got)
