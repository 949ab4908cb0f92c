"""CPU tests of the C-ABI library (no compute calls on a device).

libntc_gf256.so must load, export every symbol include/netcode/gpu.h declares, and its host-side
scalar helpers (galois_field::coefficient / multiply_size / multiply / invert) must agree with
the oracle bit for bit.
"""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols(header):
    txt = open(os.path.join(ROOT, "include", "netcode", header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ntc_gf(?:256)?_[a-z_0-9]+)\s*\(", txt)))


def test_header_symbols_match_loader_list():
    from netcode_amd import _native
    assert _declared_symbols("gpu.h") == sorted(_native.GPU_H_SYMBOLS)


def test_kernel_kind_names_match_header():
    """The timing log's kinds (NTC_GF256_K_* in gpu.h) and the names the Python mirror and
    bench.py give them (Engine.KERNEL_KINDS, indexed by value) stay in step."""
    from netcode_amd.engine import Engine
    txt = open(os.path.join(ROOT, "include", "netcode", "gpu.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    kinds = {int(v): n.lower() for n, v in re.findall(r"NTC_GF256_K_([A-Z_]+)\s*=\s*(\d+)", txt)}
    assert sorted(kinds) == list(range(len(Engine.KERNEL_KINDS)))
    alias = {"slice": "preslice"}
    assert [alias.get(kinds[i], kinds[i]) for i in sorted(kinds)] == list(Engine.KERNEL_KINDS)


def test_library_loads_and_exports(native_built):
    from netcode_amd import _native
    L = _native.load()
    for s in _declared_symbols("gpu.h"):
        assert hasattr(L, s), s
    assert b"gfx950" in L.ntc_gf256_build_info()


def test_host_helpers_match_oracle(native_built, oracle):
    from netcode_amd import _native
    L = _native.load()
    for x in range(256):
        for y in (0, 1, 2, 3, 0x53, 0xCA, 255, x):
            assert L.ntc_gf256_multiply(x, y) == oracle.gf_mul(x, y)
        if x:
            assert L.ntc_gf256_invert(x) == oracle.gf_inv(x)
    for rid, sid in [(0, 0), (1, 0), (3, 7), (31, 127), (0xFFFFFFFF, 1), (2_000_000, 8_000_000)]:
        assert L.ntc_gf256_coefficient(rid, sid) == oracle.coefficient(rid, sid)
    for size in (0, 1, 4, 6, 1024, 1500, 4096, 65535):
        for c in (0, 1, 3, 200):
            assert L.ntc_gf256_multiply_size(size, c) == oracle.multiply_size(size, c)


def test_engine_create_without_device_fails_loudly(native_built):
    import ctypes as C
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from netcode_amd import _native
    L = _native.load()
    h = C.c_void_p()
    rc = L.ntc_gf256_engine_create(0, C.byref(h))
    assert rc != 0 and not h.value
    assert L.ntc_gf256_last_error()
