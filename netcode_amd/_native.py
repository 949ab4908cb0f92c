"""Loader for the in-tree native engine ``libntc_gf256.so`` (C ABI in include/netcode/gpu.h).

There is no fallback: if the HIP library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# NTC_GF256_LIB points at an alternative build of the same library (A/B experiments only).
LIB_PATH = os.environ.get("NTC_GF256_LIB") or os.path.join(HERE, "libntc_gf256.so")

# Every symbol include/netcode/gpu.h declares (tests check the .so exports all of them).
GPU_H_SYMBOLS = [
    "ntc_gf256_engine_create", "ntc_gf256_engine_destroy", "ntc_gf256_set_mac_kind",
    "ntc_gf256_reserve", "ntc_gf256_release_retired",
    "ntc_gf256_encode_batch", "ntc_gf256_decode_batch", "ntc_gf256_decode_plan",
    "ntc_gf256_decode_apply", "ntc_gf256_region_multiply", "ntc_gf256_coef_pitch",
    "ntc_gf256_combine_batch", "ntc_gf256_coefficient",
    "ntc_gf256_multiply_size", "ntc_gf256_multiply", "ntc_gf256_invert",
    "ntc_gf256_last_error", "ntc_gf256_build_info",
    "ntc_gf256_dense_invert_batch", "ntc_gf256_dense_encode_batch", "ntc_gf256_dense_decode_batch",
    "ntc_gf256_repair_packet_bytes", "ntc_gf256_write_repairs", "ntc_gf256_write_sources",
    "ntc_gf256_read_packets", "ntc_gf256_read_packets_append", "ntc_gf256_unpack_slots", "ntc_gf256_pack_slots",
    "ntc_gf_combine_batch", "ntc_gf_region_multiply", "ntc_gf_coefficient", "ntc_gf_multiply",
    "ntc_gf_invert", "ntc_gf_multiply_size", "ntc_gf256_set_timing", "ntc_gf256_mac_time",
    "ntc_gf256_set_plan_kind", "ntc_gf256_timing_log", "ntc_gf256_timing_read", "ntc_gf256_timing_kinds",
    "ntc_gf256_gather_combine",
]

STATUS_NAMES = {0: "OK", 1: "EINVAL", 2: "ENOMEM", 3: "EDEVICE", 4: "EUNSUPPORTED"}


class NativeError(RuntimeError):
    pass


class DecodeStatus(C.Structure):
    """ntc_gf256_decode_status (include/netcode/gpu.h)."""
    _fields_ = [("state", C.c_uint8), ("nb_failed", C.c_uint8), ("nb_missing", C.c_uint16),
                ("nb_decoded", C.c_uint16), ("nb_useless", C.c_uint16),
                ("last_repair", C.c_uint16), ("pad", C.c_uint16)]


_lib = None


def load(path: str | None = None):
    """Load (once) and type the native library; raises NativeError if absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise NativeError(f"{p} not built: run `python -m netcode_amd.build` (hipcc, gfx950)")
    try:
        L = C.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime being present
        raise NativeError(f"cannot load {p}: {e}") from e
    V, P = C.c_void_p, C.c_void_p
    u32, u16, u8 = C.c_uint32, C.c_uint16, C.c_uint8
    L.ntc_gf256_engine_create.argtypes = [C.c_int, C.POINTER(V)]
    L.ntc_gf256_engine_destroy.argtypes = [V]
    L.ntc_gf256_engine_destroy.restype = None
    L.ntc_gf256_set_mac_kind.argtypes = [V, C.c_int]
    L.ntc_gf256_reserve.argtypes = [V, u32, u32, u32]
    L.ntc_gf256_release_retired.argtypes = [V]
    L.ntc_gf256_encode_batch.argtypes = [V, u32, u32, u32, u32, P, P, P, P, P, P, P, V]
    L.ntc_gf256_decode_batch.argtypes = [V, u32, u32, u32, u32, P, P, P, P, P, P, P, P, P, V]
    L.ntc_gf256_decode_plan.argtypes = [V, u32, u32, u32, P, P, P, P, P, P, P, V]
    L.ntc_gf256_decode_apply.argtypes = [V, u32, u32, u32, u32, P, P, V]
    L.ntc_gf256_region_multiply.argtypes = [V, P, P, C.c_size_t, u8, C.c_int, V]
    L.ntc_gf256_coef_pitch.argtypes = [u32]
    L.ntc_gf256_coef_pitch.restype = u32
    L.ntc_gf256_combine_batch.argtypes = [V, u32, u32, u32, u32, P, P, P, V]
    L.ntc_gf256_gather_combine.argtypes = [V, u32, P, P, u32, V]
    L.ntc_gf256_dense_invert_batch.argtypes = [V, u32, u32, P, P, P, V]
    L.ntc_gf256_dense_encode_batch.argtypes = [V, u32, u32, u32, u32, P, P, P, V]
    L.ntc_gf256_dense_decode_batch.argtypes = [V, u32, u32, u32, P, P, P, P, V]
    L.ntc_gf256_coefficient.argtypes = [u32, u32]
    L.ntc_gf256_coefficient.restype = u32
    L.ntc_gf256_multiply_size.argtypes = [u16, u32]
    L.ntc_gf256_multiply_size.restype = u16
    L.ntc_gf256_multiply.argtypes = [u8, u8]
    L.ntc_gf256_multiply.restype = u8
    L.ntc_gf256_invert.argtypes = [u8]
    L.ntc_gf256_invert.restype = u8
    L.ntc_gf256_repair_packet_bytes.argtypes = [u32, u32]
    L.ntc_gf256_repair_packet_bytes.restype = u32
    L.ntc_gf256_write_repairs.argtypes = [V, u32, u32, u32, u32, P, P, P, P, P, P, u32, P, V]
    L.ntc_gf256_write_sources.argtypes = [V, u32, u32, u32, P, P, P, P, u32, P, V]
    L.ntc_gf256_read_packets.argtypes = [V, u32, P, u32, P, u32, u32, u32, u32, u32, u32,
                                         P, P, P, P, P, P, P, V]
    L.ntc_gf256_read_packets_append.argtypes = L.ntc_gf256_read_packets.argtypes
    L.ntc_gf256_unpack_slots.argtypes = [V, u32, u32, u32, P, P, u32, P, u8, P, C.c_int, V]
    L.ntc_gf256_pack_slots.argtypes = [V, u32, u32, u32, P, P, u8, P, u32, P, V]
    L.ntc_gf256_set_timing.argtypes = [V, C.c_int]
    L.ntc_gf256_mac_time.argtypes = [V, C.c_int, C.POINTER(C.c_float)]
    L.ntc_gf256_set_plan_kind.argtypes = [V, C.c_int]
    L.ntc_gf256_timing_log.argtypes = [V, u32]
    L.ntc_gf256_timing_kinds.argtypes = [V, u32]
    L.ntc_gf256_timing_read.argtypes = [V, u32, C.POINTER(u32), P, P]
    L.ntc_gf_combine_batch.argtypes = [V, u32, u32, u32, u32, u32, P, P, P, V]
    L.ntc_gf_region_multiply.argtypes = [V, u32, P, P, C.c_size_t, u32, C.c_int, V]
    for f in ("ntc_gf_coefficient", "ntc_gf_multiply"):
        getattr(L, f).argtypes = [u32, u32, u32]
        getattr(L, f).restype = u32
    L.ntc_gf_invert.argtypes = [u32, u32]
    L.ntc_gf_invert.restype = u32
    L.ntc_gf_multiply_size.argtypes = [u32, u16, u32]
    L.ntc_gf_multiply_size.restype = u16
    L.ntc_gf256_last_error.restype = C.c_char_p
    L.ntc_gf256_build_info.restype = C.c_char_p
    for name in GPU_H_SYMBOLS:
        if not hasattr(L, name):
            raise NativeError(f"{p} does not export {name}")
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = load().ntc_gf256_last_error().decode(errors="replace")
        raise NativeError(f"{what}: {STATUS_NAMES.get(rc, rc)}: {msg}")
