"""ctypes binding of the per-packet netcode C ABI (include/netcode/c/*.h, libntc.so).

Mirrors ``ntc::encoder`` / ``ntc::decoder`` (netcode/encoder.hh, netcode/decoder.hh): packets
come out through the packet handler, decoded data through the data handler, synchronously.  The
GF(2^8) region work inside runs on the MI355X engine (libntc_gf256.so); there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(HERE, "libntc.so")

PREPARE = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_char), C.c_size_t)
SEND = C.CFUNCTYPE(None, C.c_void_p)
READ = C.CFUNCTYPE(None, C.c_void_p, C.POINTER(C.c_char), C.c_size_t)


class PacketHandler(C.Structure):
    _fields_ = [("context", C.c_void_p), ("prepare_packet", PREPARE), ("send_packet", SEND)]


class DataHandler(C.Structure):
    _fields_ = [("context", C.c_void_p), ("read_data", READ)]


class Error(C.Structure):
    _fields_ = [("type", C.c_int), ("message", C.c_char_p)]


ERRORS = {0: "no_error", 1: "unknown_error", 2: "no_memory", 3: "packet_type_error",
          4: "overflow_error"}


class NtcError(RuntimeError):
    def __init__(self, kind: str, message: str = ""):
        super().__init__(f"{kind}: {message}" if message else kind)
        self.kind = kind


def header_symbols() -> list[str]:
    """Every ntc_* function declared by include/netcode/c/*.h."""
    out = set()
    d = os.path.join(ROOT, "include", "netcode", "c")
    for f in os.listdir(d):
        txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(d, f)).read(), flags=re.S)
        out.update(re.findall(r"\b(ntc_[a-z_0-9]+)\s*\(", txt))
    return sorted(out)


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"{LIB_PATH} not built: run `python -m netcode_amd.build`")
    L = C.CDLL(LIB_PATH)
    P, S, u16, u8 = C.c_void_p, C.c_size_t, C.c_uint16, C.c_uint8
    E = C.POINTER(Error)
    sig = {
        "ntc_new_data": (P, [u16]), "ntc_new_data_from": (P, [C.c_char_p, u16]),
        "ntc_delete_data": (None, [P]), "ntc_data_buffer": (P, [P]),
        "ntc_data_get_size": (u16, [P]), "ntc_data_resize": (None, [P, u16, E]),
        "ntc_new_packet": (P, [u16]), "ntc_new_packet_from": (P, [C.c_char_p, u16]),
        "ntc_delete_packet": (None, [P]), "ntc_packet_buffer": (P, [P]),
        "ntc_packet_get_size": (u16, [P]), "ntc_packet_resize": (None, [P, u16, E]),
        "ntc_new_encoder": (P, [u8, PacketHandler]), "ntc_delete_encoder": (None, [P]),
        "ntc_encoder_add_data": (None, [P, P, E]), "ntc_encoder_add_packet": (S, [P, P, E]),
        "ntc_encoder_generate_repair": (None, [P, E]), "ntc_encoder_window": (S, [P]),
        "ntc_encoder_set_code_type": (None, [P, C.c_int]), "ntc_encoder_set_rate": (None, [P, S]),
        "ntc_encoder_set_window_size": (None, [P, S]), "ntc_encoder_set_adaptive": (None, [P, C.c_bool]),
        "ntc_new_decoder": (P, [u8, C.c_int, PacketHandler, DataHandler]),
        "ntc_delete_decoder": (None, [P]), "ntc_decoder_add_packet": (S, [P, P, E]),
        "ntc_decoder_generate_ack": (None, [P, E]), "ntc_decoder_set_ack_period": (None, [P, S]),
        "ntc_decoder_set_ack_nb_packets": (None, [P, u16]),
        "ntc_encoder_counter": (S, [P, C.c_int]), "ntc_decoder_counter": (S, [P, C.c_int]),
        "ntc_new_batch": (P, []), "ntc_delete_batch": (None, [P]),
        "ntc_encoder_set_batch": (None, [P, P, E]), "ntc_decoder_set_batch": (None, [P, P, E]),
        "ntc_batch_flush": (None, [P, E]),
        "ntc_batch_pending": (S, [P]), "ntc_batch_set_eager": (None, [P, C.c_int]),
        "ntc_batch_set_async": (None, [P, C.c_int]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(err: Error):
    if err.type != 0:
        raise NtcError(ERRORS.get(err.type, str(err.type)),
                       err.message.decode(errors="replace") if err.message else "")


class _Collector:
    """Packet handler that concatenates prepare_packet pieces into whole packets."""

    def __init__(self):
        self.packets: list[bytes] = []
        self._cur = bytearray()
        self._p = PREPARE(lambda ctx, data, n: self._cur.extend(C.string_at(data, n)))
        self._s = SEND(self._end)
        self.handler = PacketHandler(None, self._p, self._s)

        self.on_packet = None         # optional hook, called with each finished packet

    def _end(self, ctx):
        pkt = bytes(self._cur)
        self.packets.append(pkt)
        self._cur = bytearray()
        if self.on_packet is not None:
            self.on_packet(pkt)


def _packet(L, pkt: bytes):
    p = L.ntc_new_packet_from(bytes(pkt), len(pkt)) if pkt else L.ntc_new_packet(0)
    if not p:
        raise MemoryError
    return p


class Encoder:
    COUNTERS = ["nb_sent_repairs", "nb_sent_sources", "nb_received_acks", "rate", "window"]

    def __init__(self, galois_field_size: int = 8):
        self.L = load()
        self._out = _Collector()
        self.h = self.L.ntc_new_encoder(galois_field_size, self._out.handler)
        if not self.h:
            raise NtcError("unknown_error", "ntc_new_encoder failed (no MI355X engine?)")

    @property
    def packets(self):
        return self._out.packets

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ntc_delete_encoder(self.h)
            self.h = None

    def add_data(self, data: bytes):
        d = self.L.ntc_new_data_from(bytes(data), len(data)) if data else self.L.ntc_new_data(0)
        err = Error(0, None)
        try:
            self.L.ntc_encoder_add_data(self.h, d, C.byref(err))
        finally:
            self.L.ntc_delete_data(d)
        _check(err)

    def add_packet(self, pkt: bytes) -> int:
        p = _packet(self.L, pkt)
        err = Error(0, None)
        try:
            n = self.L.ntc_encoder_add_packet(self.h, p, C.byref(err))
        finally:
            self.L.ntc_delete_packet(p)
        _check(err)
        return n

    def generate_repair(self):
        err = Error(0, None)
        self.L.ntc_encoder_generate_repair(self.h, C.byref(err))
        _check(err)

    def set_rate(self, r):
        self.L.ntc_encoder_set_rate(self.h, r)

    def set_window_size(self, s):
        self.L.ntc_encoder_set_window_size(self.h, s)

    def set_code_type(self, systematic: bool):
        self.L.ntc_encoder_set_code_type(self.h, 0 if systematic else 1)

    def set_adaptive(self, a: bool):
        self.L.ntc_encoder_set_adaptive(self.h, bool(a))

    def set_batch(self, batch: "Batch | None"):
        """Attach to an online batching adaptor (None detaches; flushes the current batch)."""
        err = Error(0, None)
        self.L.ntc_encoder_set_batch(self.h, batch.h if batch is not None else None, C.byref(err))
        _check(err)
        self._batch = batch          # keep the batch alive while attached

    def __getattr__(self, name):
        if name in Encoder.COUNTERS:
            return self.L.ntc_encoder_counter(self.h, Encoder.COUNTERS.index(name))
        raise AttributeError(name)


class Batch:
    """ntc_batch_t (netcode/c/ext.h): attached encoders' packets are queued until flush(), which
    computes every pending repair in one GPU launch per field size and emits in production order."""

    def __init__(self, eager: bool = False, asynchronous: bool = False):
        self.L = load()
        self.h = self.L.ntc_new_batch()
        if not self.h:
            raise MemoryError
        if eager:
            self.L.ntc_batch_set_eager(self.h, 1)
        if asynchronous:          # a flush delivers the previous flush's events, returns at once
            self.L.ntc_batch_set_async(self.h, 1)

    def flush(self):
        err = Error(0, None)
        self.L.ntc_batch_flush(self.h, C.byref(err))
        _check(err)

    @property
    def pending(self) -> int:
        return self.L.ntc_batch_pending(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ntc_delete_batch(self.h)
            self.h = None


class Decoder:
    COUNTERS = ["nb_decoded", "nb_failed_full_decodings", "nb_missing_sources",
                "nb_received_repairs", "nb_received_sources", "nb_sent_acks",
                "nb_useless_repairs", "nb_pending_repairs"]

    def __init__(self, galois_field_size: int = 8, in_order: bool = True):
        self.L = load()
        self._out = _Collector()
        self.data: list[bytes] = []
        self.aligned = True
        self._r = READ(self._read)
        self._dh = DataHandler(None, self._r)
        self.h = self.L.ntc_new_decoder(galois_field_size, 0 if in_order else 1, self._out.handler,
                                        self._dh)
        if not self.h:
            raise NtcError("unknown_error", "ntc_new_decoder failed (no MI355X engine?)")

    def _read(self, ctx, data, n):
        self.aligned &= (C.cast(data, C.c_void_p).value or 0) % 16 == 0
        self.data.append(C.string_at(data, n))

    @property
    def packets(self):
        return self._out.packets

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ntc_delete_decoder(self.h)
            self.h = None

    def add_packet(self, pkt: bytes) -> int:
        p = _packet(self.L, pkt)
        err = Error(0, None)
        try:
            n = self.L.ntc_decoder_add_packet(self.h, p, C.byref(err))
        finally:
            self.L.ntc_delete_packet(p)
        _check(err)
        return n

    def set_batch(self, batch: "Batch | None"):
        """Attach to an online batching adaptor (None detaches; flushes the current batch)."""
        err = Error(0, None)
        self.L.ntc_decoder_set_batch(self.h, batch.h if batch is not None else None, C.byref(err))
        _check(err)
        self._batch = batch

    def generate_ack(self):
        err = Error(0, None)
        self.L.ntc_decoder_generate_ack(self.h, C.byref(err))
        _check(err)

    def set_ack_period_ms(self, ms):
        self.L.ntc_decoder_set_ack_period(self.h, ms)

    def set_ack_nb_packets(self, n):
        self.L.ntc_decoder_set_ack_nb_packets(self.h, n)

    def __getattr__(self, name):
        if name in Decoder.COUNTERS:
            return self.L.ntc_decoder_counter(self.h, Decoder.COUNTERS.index(name))
        raise AttributeError(name)
