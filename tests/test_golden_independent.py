"""An independent pin of the committed golden fixtures (tests/golden/*.npz).

make_golden.py writes the fixtures from the oracle, so checking the oracle against them only
catches regressions.  Here they are re-derived WITHOUT the oracle: GF(2^8) from gf-complete's
default polynomial 0x11D (galois_field.hh:35-44) by log / exp tables built in numpy, the repair
coefficients from galois_field.hh:143-158, repair symbols as the XOR of coefficient x source
(encoder.hh: a repair is the linear combination of the window's sources) and repair sizes from
multiply_size (galois_field.hh:96-120: for w = 8 the two bytes of the u16 are multiplied as a
region).  Decoded outputs are checked for what the bytes must be whatever the elimination order:
every source the decoder reports (non-zero length) equals the source that was sent, and only
lost sources may be missing.  CPU only."""
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ["gen_k16_r4_loss25", "gen_k32_r8_ragged"]


def _tables():
    exp = np.zeros(512, np.int64)
    log = np.zeros(256, np.int64)
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    exp[255:510] = exp[0:255]
    return exp, log


EXP, LOG = _tables()


def gf_mul_region(c, v):
    """c * v for a uint8 array v (numpy, log / exp tables)."""
    if c == 0:
        return np.zeros_like(v)
    out = EXP[(LOG[v.astype(np.int64)] + LOG[c]) % 255].astype(np.uint8)
    out[v == 0] = 0
    return out


def coefficient(rid, sid):
    """galois_field.hh:143-158, w = 8 (uint32 arithmetic)."""
    return ((((rid + 1) + (sid + 1)) * (rid + 1)) & 0xFFFFFFFF) % 255 + 1


def multiply_size(size, c):
    if size == 0 or c == 0:
        return 0
    b = np.array([size & 0xFF, size >> 8], np.uint8)
    m = gf_mul_region(c, b)
    return int(m[0]) | (int(m[1]) << 8)


def _clmul_reduce(a, b):
    r = 0
    for i in range(8):
        if (b >> i) & 1:
            r ^= a << i
    for i in range(14, 7, -1):
        if (r >> i) & 1:
            r ^= 0x11D << (i - 8)
    return r


def test_field_tables():
    # 2 generates GF(2^8) under 0x11D, and the table product equals the carry-less product
    # reduced by 0x11D for every pair
    assert sorted(EXP[:255].tolist()) == list(range(1, 256))
    v = np.arange(256, dtype=np.uint8)
    for a in range(256):
        assert gf_mul_region(a, v).tolist() == [_clmul_reduce(a, b) for b in range(256)], a


@pytest.mark.parametrize("name", NAMES)
def test_golden_repairs_independent(name):
    z = np.load(os.path.join(HERE, name + ".npz"))
    src, lens, sid, rid = z["src"], z["src_len"], z["sid_base"], z["rid_base"]
    G, k, stride = src.shape
    r = z["rep"].shape[1]
    for g in range(0, G, max(1, G // 40)):            # a spread of generations (pure numpy)
        for j in range(r):
            R = int(rid[g]) + j
            acc = np.zeros(stride, np.uint8)
            size = 0
            for i in range(k):
                c = coefficient(R, int(sid[g]) + i)
                acc ^= gf_mul_region(c, src[g, i])
                size ^= multiply_size(int(lens[g, i]), c)
            assert (acc == z["rep"][g, j]).all(), (name, g, j)
            assert size == int(z["rep_size"][g, j]), (name, g, j)


@pytest.mark.parametrize("name", NAMES)
def test_golden_decodes_are_the_sources(name):
    z = np.load(os.path.join(HERE, name + ".npz"))
    src, lens, out, olen = z["src"], z["src_len"], z["out"], z["out_len"]
    smask, rmask = z["src_mask"], z["rep_mask"]
    G, k, _ = src.shape
    recovered = 0
    for g in range(G):
        for i in range(k):
            if olen[g, i]:
                assert olen[g, i] == lens[g, i] and (out[g, i] == src[g, i]).all(), (name, g, i)
                recovered += int(smask[g, i] == 0)
            else:
                assert smask[g, i] == 0 or lens[g, i] == 0, (name, g, i)   # only lost ones missing
        # never more lost sources rebuilt than repairs received
        lost_back = int(((smask[g] == 0) & (olen[g] > 0)).sum())
        assert lost_back <= int(rmask[g].sum()), (name, g)
    assert recovered > 0
