"""ctypes binding of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module. It
restates ahamez/netcode's GF(2^8) path (see ntc_oracle.c for per-function reference citations)
and is never used by the product package ``netcode_amd``.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libntc_oracle.so")
_lib = None


class DecodeStatus(C.Structure):
    _fields_ = [("state", C.c_uint8), ("nb_failed", C.c_uint8), ("nb_missing", C.c_uint16),
                ("nb_decoded", C.c_uint16), ("nb_useless", C.c_uint16),
                ("last_repair", C.c_uint16), ("pad", C.c_uint16)]


DECODE_STATUS_DTYPE = np.dtype([("state", "u1"), ("nb_failed", "u1"), ("nb_missing", "<u2"),
                                ("nb_decoded", "<u2"), ("nb_useless", "<u2"),
                                ("last_repair", "<u2"), ("pad", "<u2")])

EMIT = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)
DELIVER = C.CFUNCTYPE(None, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint8), C.c_size_t)


def build() -> str:
    """Compile the oracle (gcc) in place; idempotent."""
    src = os.path.join(_HERE, "ntc_oracle.c")
    if (not os.path.exists(_LIB)) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = C.CDLL(_LIB)
        P = C.c_void_p
        u8p, u16p, u32p = C.POINTER(C.c_uint8), C.POINTER(C.c_uint16), C.POINTER(C.c_uint32)
        L.or_gf_mul.restype = C.c_uint8
        L.or_gf_mul.argtypes = [C.c_uint8, C.c_uint8]
        L.or_gf_inv.restype = C.c_uint32
        L.or_gf_inv.argtypes = [C.c_uint32]
        L.or_coefficient.restype = C.c_uint32
        L.or_coefficient.argtypes = [C.c_uint32, C.c_uint32]
        L.or_multiply_size.restype = C.c_uint16
        L.or_multiply_size.argtypes = [C.c_uint16, C.c_uint32]
        L.or_region_mul.argtypes = [P, P, C.c_size_t, C.c_uint32]
        L.or_region_muladd.argtypes = [P, P, C.c_size_t, C.c_uint32]
        L.or_fw_mul.restype = C.c_uint32
        L.or_fw_mul.argtypes = [C.c_int, C.c_uint32, C.c_uint32]
        L.or_fw_inv.restype = C.c_uint32
        L.or_fw_inv.argtypes = [C.c_int, C.c_uint32]
        L.or_fw_coefficient.restype = C.c_uint32
        L.or_fw_coefficient.argtypes = [C.c_int, C.c_uint32, C.c_uint32]
        L.or_fw_region.argtypes = [C.c_int, P, P, C.c_size_t, C.c_uint32, C.c_int]
        L.or_fw_multiply_size.restype = C.c_uint16
        L.or_fw_multiply_size.argtypes = [C.c_int, C.c_uint16, C.c_uint32]
        L.or_encoder_set_field.argtypes = [P, C.c_int]
        L.or_decoder_set_field.argtypes = [P, C.c_int]
        L.or_region_muladd_simd.argtypes = [P, P, C.c_size_t, C.c_uint8]
        L.or_invert.restype = C.c_long
        L.or_invert.argtypes = [P, P, C.c_size_t]
        L.or_dense_encode.argtypes = [C.c_uint32, C.c_uint32, C.c_size_t, P, P, P]
        L.or_dense_encode.restype = None
        L.or_dense_decode.argtypes = [C.c_uint32, C.c_size_t, P, P, P, P]
        L.or_dense_decode.restype = C.c_long
        L.or_encode_generation.argtypes = [C.c_uint32] * 3 + [P, P, C.c_uint32, C.c_uint32,
                                                              P, P, P]
        L.or_encode_batch.argtypes = [C.c_uint32] * 4 + [P, P, P, P, P, P, C.c_int, C.c_int]
        L.or_decode_batch.argtypes = [C.c_uint32] * 4 + [P] * 10 + [C.c_int, C.c_int]
        L.or_end_to_end.restype = C.c_int
        L.or_end_to_end.argtypes = [C.c_uint32, P]
        L.or_encoder_new.restype = P
        L.or_encoder_new.argtypes = [EMIT, P]
        L.or_encoder_free.argtypes = [P]
        L.or_encoder_set_rate.argtypes = [P, C.c_size_t]
        L.or_encoder_set_window_size.argtypes = [P, C.c_size_t]
        L.or_encoder_set_code_type.argtypes = [P, C.c_int]
        L.or_encoder_set_adaptive.argtypes = [P, C.c_int]
        L.or_encoder_add_data.argtypes = [P, P, C.c_uint16]
        L.or_encoder_add_packet.restype = C.c_long
        L.or_encoder_add_packet.argtypes = [P, P, C.c_size_t]
        L.or_encoder_generate_repair.argtypes = [P]
        for n in ("window", "rate", "nb_sent_repairs", "nb_sent_sources", "nb_received_acks"):
            f = getattr(L, "or_encoder_" + n)
            f.restype = C.c_size_t
            f.argtypes = [P]
        L.or_decoder_new.restype = P
        L.or_decoder_new.argtypes = [C.c_int, EMIT, P, DELIVER, P]
        L.or_decoder_free.argtypes = [P]
        L.or_decoder_add_packet.restype = C.c_long
        L.or_decoder_add_packet.argtypes = [P, P, C.c_size_t]
        L.or_decoder_generate_ack.argtypes = [P]
        L.or_decoder_set_ack_nb_packets.argtypes = [P, C.c_uint16]
        L.or_decoder_set_ack_period_ms.argtypes = [P, C.c_long]
        L.or_decoder_counter.restype = C.c_size_t
        L.or_decoder_counter.argtypes = [P, C.c_int]
        L.or_have_avx2.restype = C.c_int
        L.or_have_gfni.restype = C.c_int
        L.or_pp_bench.argtypes = [C.c_uint32] * 6 + [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
        L.or_set_simd.argtypes = [C.c_int]
        L.or_write_repair_packet.restype = C.c_size_t
        L.or_write_repair_packet.argtypes = [C.c_uint32, P, C.c_uint16, P, C.c_size_t, C.c_uint16, P]
        L.or_write_source_packet.restype = C.c_size_t
        L.or_write_source_packet.argtypes = [C.c_uint32, P, C.c_uint16, P]
        L.or_read_packet_into.restype = C.c_int
        L.or_read_packet_into.argtypes = [P, C.c_size_t] + [C.c_uint32] * 6 + [P] * 6
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


# --------------------------------------------------------------------------- scalar helpers
def gf_mul(a: int, b: int) -> int:
    return lib().or_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().or_gf_inv(a)


def coefficient(rid: int, sid: int) -> int:
    return lib().or_coefficient(rid & 0xFFFFFFFF, sid & 0xFFFFFFFF)


def multiply_size(size: int, c: int) -> int:
    return lib().or_multiply_size(size, c)


def mul_table() -> np.ndarray:
    """256x256 product table (0x11D)."""
    t = np.zeros((256, 256), np.uint8)
    L = lib()
    for a in range(256):
        src = np.arange(256, dtype=np.uint8)
        L.or_region_mul(_p(src), _p(t[a]), 256, a)
    return t


def invert(mat_colmajor: np.ndarray):
    """Returns (failure_index or None, inverse col-major u32)."""
    n = int(round(np.sqrt(mat_colmajor.size)))
    m = np.ascontiguousarray(mat_colmajor, dtype=np.uint32).copy()
    inv = np.zeros(n * n, np.uint32)
    r = lib().or_invert(_p(m), _p(inv), n)
    return (None if r < 0 else int(r)), inv


def dense_encode(mat: np.ndarray, src: np.ndarray) -> np.ndarray:
    """rep[j] = sum_i mat[j][i] * src[i]; mat [r][k] u8, src [k][stride]."""
    r, k = mat.shape
    stride = src.shape[1]
    rep = np.zeros((r, stride), np.uint8)
    lib().or_dense_encode(k, r, stride, _p(np.ascontiguousarray(mat, np.uint8)),
                          _p(np.ascontiguousarray(src, np.uint8)), _p(rep))
    return rep


def dense_decode(mat: np.ndarray, rep: np.ndarray):
    """(ok, out = mat^-1 rep, inv) for one dense n x n system."""
    n = mat.shape[0]
    stride = rep.shape[1]
    out = np.zeros((n, stride), np.uint8)
    inv = np.zeros((n, n), np.uint8)
    f = lib().or_dense_decode(n, stride, _p(np.ascontiguousarray(mat, np.uint8)),
                              _p(np.ascontiguousarray(rep, np.uint8)), _p(out), _p(inv))
    return f < 0, out, inv


# --------------------------------------------------------------------------- batch forms
def encode_batch(src, src_len, k, r, sid_base=None, rid_base=None, simd=False, threads=1):
    G, kk, stride = src.shape
    assert kk == k
    rep = np.zeros((G, r, stride), np.uint8)
    rep_size = np.zeros((G, r), np.uint16)
    lib().or_encode_batch(G, k, r, stride, _p(np.ascontiguousarray(src)),
                          _p(np.ascontiguousarray(src_len, dtype=np.uint16)),
                          _p(None if sid_base is None else np.ascontiguousarray(sid_base, np.uint32)),
                          _p(None if rid_base is None else np.ascontiguousarray(rid_base, np.uint32)),
                          _p(rep), _p(rep_size), int(simd), int(threads))
    return rep, rep_size


def decode_batch(src, src_len, src_mask, rep, rep_size, rep_mask, sid_base=None, rid_base=None,
                 rep_len=None, threads=1):
    """Returns (src_out, src_len_out, status[G]) -- inputs are not modified."""
    G, k, stride = src.shape
    r = rep.shape[1]
    s = np.ascontiguousarray(src).copy()
    sl = np.ascontiguousarray(src_len, dtype=np.uint16).copy()
    st = np.zeros(G, DECODE_STATUS_DTYPE)
    lib().or_decode_batch(G, k, r, stride, _p(s), _p(sl),
                          _p(np.ascontiguousarray(src_mask, np.uint8)),
                          _p(np.ascontiguousarray(rep)), _p(np.ascontiguousarray(rep_size, np.uint16)),
                          _p(None if rep_len is None else np.ascontiguousarray(rep_len, np.uint16)),
                          _p(np.ascontiguousarray(rep_mask, np.uint8)),
                          _p(None if sid_base is None else np.ascontiguousarray(sid_base, np.uint32)),
                          _p(None if rid_base is None else np.ascontiguousarray(rid_base, np.uint32)),
                          _p(st), 0, int(threads))
    return s, sl, st


# --------------------------------------------------------------------------- GF(2^w)
def fw_mul(w: int, a: int, b: int) -> int:
    return lib().or_fw_mul(w, a & 0xFFFFFFFF, b & 0xFFFFFFFF)


def fw_inv(w: int, a: int) -> int:
    return lib().or_fw_inv(w, a & 0xFFFFFFFF)


def fw_coefficient(w: int, rid: int, sid: int) -> int:
    return lib().or_fw_coefficient(w, rid & 0xFFFFFFFF, sid & 0xFFFFFFFF)


def fw_multiply_size(w: int, size: int, c: int) -> int:
    return lib().or_fw_multiply_size(w, size, c & 0xFFFFFFFF)


def fw_region(w: int, src: np.ndarray, dst: np.ndarray, c: int, add: bool) -> np.ndarray:
    """dst (copy) = c*src (+ dst) over len(src) bytes in GF(2^w)."""
    src = np.ascontiguousarray(src, np.uint8)
    out = np.ascontiguousarray(dst, np.uint8).copy()
    lib().or_fw_region(w, _p(src), _p(out), src.size, c & 0xFFFFFFFF, int(add))
    return out


# --------------------------------------------------------------------------- wire format
def write_repair_packet(rid, sym, ids, esz) -> bytes:
    """packetizer.hh:90-122: one repair packet (sym = the symbol bytes, ids ascending)."""
    sym = np.ascontiguousarray(sym, np.uint8)
    ids = np.ascontiguousarray(ids, np.uint32)
    out = np.zeros(32 + 2 * sym.size + 3 * ids.size, np.uint8)
    n = lib().or_write_repair_packet(rid & 0xFFFFFFFF, _p(sym), sym.size, _p(ids), ids.size, esz,
                                     _p(out))
    return out[:n].tobytes()


def write_source_packet(sid, data) -> bytes:
    """packetizer.hh:165-183: one source packet."""
    data = np.ascontiguousarray(data, np.uint8)
    out = np.zeros(16 + data.size, np.uint8)
    n = lib().or_write_source_packet(sid & 0xFFFFFFFF, _p(data), data.size, _p(out))
    return out[:n].tobytes()


def read_packets(pkts, G, k, r, stride, sid0=0, rid0=0):
    """Ingest wire packets (list of bytes) into a fresh batch layout; returns (src, src_len,
    src_mask, rep, rep_size, rep_mask, status[npkts]) -- the specification of
    ntc_gf256_read_packets."""
    src = np.zeros((G, k, stride), np.uint8)
    src_len = np.zeros((G, k), np.uint16)
    src_mask = np.zeros((G, k), np.uint8)
    rep = np.zeros((G, r, stride), np.uint8)
    rep_size = np.zeros((G, r), np.uint16)
    rep_mask = np.zeros((G, r), np.uint8)
    st = np.zeros(len(pkts), np.uint8)
    L = lib()
    for i, p in enumerate(pkts):
        b = np.frombuffer(p, np.uint8) if len(p) else np.zeros(1, np.uint8)
        st[i] = L.or_read_packet_into(_p(b), len(p), G, k, r, stride, sid0 & 0xFFFFFFFF,
                                      rid0 & 0xFFFFFFFF, _p(src), _p(src_len), _p(src_mask),
                                      _p(rep), _p(rep_size), _p(rep_mask))
    return src, src_len, src_mask, rep, rep_size, rep_mask, st


def end_to_end(nb_packets: int):
    out = np.zeros(7, np.uint64)
    rc = lib().or_end_to_end(nb_packets, _p(out))
    keys = ["sent", "lost", "received_repairs", "received_sources", "useless_repairs", "decoded",
            "handled_data"]
    return rc, dict(zip(keys, (int(x) for x in out)))


# --------------------------------------------------------------------------- streaming objects
class Encoder:
    """Packet-level restatement of ntc::encoder (encoder.hh); packets collected in .packets."""

    def __init__(self, galois_field_size: int = 8):
        self.packets: list[bytes] = []
        self._cb = EMIT(lambda ctx, p, n: self.packets.append(C.string_at(p, n)))
        self.h = lib().or_encoder_new(self._cb, None)
        lib().or_encoder_set_field(self.h, galois_field_size)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_encoder_free(self.h)
            self.h = None

    def add_data(self, data: bytes):
        buf = np.frombuffer(bytes(data), np.uint8).copy() if data else np.zeros(1, np.uint8)
        lib().or_encoder_add_data(self.h, _p(buf), len(data))

    def add_packet(self, pkt: bytes) -> int:
        buf = np.frombuffer(bytes(pkt), np.uint8).copy()
        return lib().or_encoder_add_packet(self.h, _p(buf), len(pkt))

    def generate_repair(self):
        lib().or_encoder_generate_repair(self.h)

    def set_rate(self, r):
        lib().or_encoder_set_rate(self.h, r)

    def set_window_size(self, s):
        lib().or_encoder_set_window_size(self.h, s)

    def set_code_type(self, systematic: bool):
        lib().or_encoder_set_code_type(self.h, int(systematic))

    def set_adaptive(self, a: bool):
        lib().or_encoder_set_adaptive(self.h, int(a))

    @property
    def window(self):
        return lib().or_encoder_window(self.h)

    @property
    def rate(self):
        return lib().or_encoder_rate(self.h)

    @property
    def nb_sent_repairs(self):
        return lib().or_encoder_nb_sent_repairs(self.h)

    @property
    def nb_sent_sources(self):
        return lib().or_encoder_nb_sent_sources(self.h)


class Decoder:
    """Packet-level restatement of ntc::decoder (decoder.hh); deliveries in .data."""

    COUNTERS = ["nb_decoded", "nb_failed_full_decodings", "nb_missing_sources",
                "nb_received_repairs", "nb_received_sources", "nb_sent_acks",
                "nb_useless_repairs", "nb_pending_repairs"]

    def __init__(self, in_order: bool = True, galois_field_size: int = 8):
        self.packets: list[bytes] = []
        self.data: list[tuple[int, bytes]] = []
        self._ecb = EMIT(lambda ctx, p, n: self.packets.append(C.string_at(p, n)))
        self._dcb = DELIVER(lambda ctx, i, p, n: self.data.append((i, C.string_at(p, n))))
        self.h = lib().or_decoder_new(int(in_order), self._ecb, None, self._dcb, None)
        lib().or_decoder_set_field(self.h, galois_field_size)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_decoder_free(self.h)
            self.h = None

    def add_packet(self, pkt: bytes) -> int:
        buf = np.frombuffer(bytes(pkt), np.uint8).copy()
        return lib().or_decoder_add_packet(self.h, _p(buf), len(pkt))

    def generate_ack(self):
        lib().or_decoder_generate_ack(self.h)

    def set_ack_nb_packets(self, n):
        lib().or_decoder_set_ack_nb_packets(self.h, n)

    def set_ack_period_ms(self, ms):
        lib().or_decoder_set_ack_period_ms(self.h, ms)

    def __getattr__(self, name):
        if name in Decoder.COUNTERS:
            return lib().or_decoder_counter(self.h, Decoder.COUNTERS.index(name))
        raise AttributeError(name)


# --------------------------------------------------------------------------- loss models
class _BurstS(C.Structure):
    _fields_ = [("state", C.c_uint32), ("bad", C.c_int), ("good_th", C.c_uint),
                ("bad_th", C.c_uint)]


class Burst:
    """tools/loss/burst.hh (libstdc++ minstd_rand0 + uniform_int_distribution{1,100})."""

    def __init__(self, good: int, bad: int):
        self.s = _BurstS()
        L = lib()
        L.or_burst_init.argtypes = [C.POINTER(_BurstS), C.c_uint, C.c_uint]
        L.or_burst_next.argtypes = [C.POINTER(_BurstS)]
        L.or_burst_next.restype = C.c_int
        L.or_burst_init(C.byref(self.s), good, bad)

    def __call__(self) -> bool:
        return bool(lib().or_burst_next(C.byref(self.s)))
