"""Host-side mirror of netcode's coding interface over the MI355X engine.

Python surface (device tensors in, device tensors out; the GF work runs in libntc_gf256.so):

* :class:`GaloisField`  -- ``ntc::detail::galois_field`` (netcode/detail/galois_field.hh:18-167):
  ``coefficient``, ``multiply`` / ``multiply_add`` (device regions), ``multiply_size``,
  scalar ``multiply`` / ``invert`` for w in {4, 8, 16, 32}; :func:`combine` batched GF(2^w)
  combinations.
* :class:`BatchEncoder` -- ``ntc::detail::encoder`` (netcode/detail/encoder.cc:15-64) applied to
  G independent generations of k sources -> r repairs each.
* :class:`BatchDecoder` -- ``ntc::detail::decoder`` (netcode/detail/decoder.cc:54-152, 412-566)
  applied to G generations whose received sources then received repairs arrive in id order.

Every call enqueues on torch's current HIP stream for the tensors' device.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _native

STATUS_DTYPE = np.dtype([("state", "u1"), ("nb_failed", "u1"), ("nb_missing", "<u2"),
                         ("nb_decoded", "<u2"), ("nb_useless", "<u2"),
                         ("last_repair", "<u2"), ("pad", "<u2")])
STATUS_BYTES = STATUS_DTYPE.itemsize  # 12

DECODED, NOTHING_MISSING, NOT_ENOUGH_REPAIRS, SINGULAR = 0, 1, 2, 3


def _ptr(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


def _stream(dev: torch.device):
    return torch.cuda.current_stream(dev).cuda_stream


def _require(t: torch.Tensor, name: str, dtype, shape, dev):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device != dev:
        raise ValueError(f"{name} must live on {dev}, got {t.device}")
    if t.dtype not in dtype:
        raise TypeError(f"{name} must have dtype {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


_U8 = (torch.uint8,)
_U16 = (torch.int16, torch.uint16)
_U32 = (torch.int32, torch.uint32)


class Engine:
    """One native engine per HIP device (ntc_gf256_engine_create)."""

    _per_device: dict[int, "Engine"] = {}

    def __init__(self, device: int | torch.device = 0):
        L = _native.load()
        dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if dev.type != "cuda":
            raise ValueError("the GF(256) engine runs on a HIP device")
        self.device = torch.device("cuda", dev.index if dev.index is not None else 0)
        h = _native.C.c_void_p()
        _native.check(L.ntc_gf256_engine_create(self.device.index, _native.C.byref(h)),
                      "ntc_gf256_engine_create")
        self._h = h
        self._L = L

    @classmethod
    def get(cls, device: int | torch.device = 0) -> "Engine":
        idx = device if isinstance(device, int) else (torch.device(device).index or 0)
        if idx not in cls._per_device:
            cls._per_device[idx] = Engine(idx)
        return cls._per_device[idx]

    def close(self):
        if getattr(self, "_h", None):
            self._L.ntc_gf256_engine_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown ordering
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    MAC_KINDS = {"auto": 0, "perm": 1, "bitslice": 2, "grouped": 3, "paired": 4}

    def set_mac_kind(self, kind: str = "auto"):
        """Select the region-MAC formulation (ntc_gf256_set_mac_kind); results are identical."""
        _native.check(self._L.ntc_gf256_set_mac_kind(self._h, Engine.MAC_KINDS[kind]),
                      "ntc_gf256_set_mac_kind")

    PLAN_KINDS = {"auto": 0, "wave": 1, "lds": 2, "big": 3}

    def set_plan_kind(self, kind: str = "auto"):
        """Select the decode-plan kernel (ntc_gf256_set_plan_kind); results are identical."""
        _native.check(self._L.ntc_gf256_set_plan_kind(self._h, Engine.PLAN_KINDS[kind]),
                      "ntc_gf256_set_plan_kind")

    KERNEL_KINDS = ("encode_prep", "encode_mac", "decode_plan", "plan_rows", "decode_mac",
                    "bj_offsets", "dense", "other", "preslice")

    def timing_log(self, capacity: int, kinds=None):
        """Bracket each of the next `capacity` kernel launches with HIP events (0 = off);
        `kinds` (names of KERNEL_KINDS) restricts the log to those kernels (None = all)."""
        self.timing_kinds(kinds)
        _native.check(self._L.ntc_gf256_timing_log(self._h, int(capacity)), "ntc_gf256_timing_log")

    def timing_kinds(self, kinds=None):
        """Restrict the running log to `kinds` from now on (None = all); logged entries stay."""
        mask = 0xFFFFFFFF if kinds is None else sum(1 << Engine.KERNEL_KINDS.index(k) for k in kinds)
        _native.check(self._L.ntc_gf256_timing_kinds(self._h, mask), "ntc_gf256_timing_kinds")

    def timing_read(self, max_entries: int = 1 << 16):
        """[(kernel kind name, ms)] of the logged launches, in launch order (waits for them)."""
        import ctypes as C
        kinds = (C.c_uint32 * max_entries)()
        ms = (C.c_float * max_entries)()
        n = C.c_uint32()
        _native.check(self._L.ntc_gf256_timing_read(self._h, max_entries, C.byref(n),
                                                     C.addressof(kinds), C.addressof(ms)),
                      "ntc_gf256_timing_read")
        return [(Engine.KERNEL_KINDS[kinds[i]], float(ms[i])) for i in range(min(n.value, max_entries))]

    def reserve(self, G: int, k: int, r: int):
        _native.check(self._L.ntc_gf256_reserve(self._h, G, k, r), "ntc_gf256_reserve")


class GaloisField:
    """``ntc::detail::galois_field`` (galois_field.hh:18-167) for w in {4, 8, 16, 32}.

    GF(2^8) uses the engine's dedicated kernels and tables (ntc_gf256_*); the other sizes the
    generic packed shift-and-add kernels (ntc_gf_*, gf-complete's default polynomials)."""

    SIZES = (4, 8, 16, 32)

    def __init__(self, w: int = 8, device: int | torch.device = 0):
        if w not in GaloisField.SIZES:
            raise ValueError("galois field size must be 4, 8, 16 or 32")
        self.w = w
        self._L = _native.load()
        self._dev = device

    def size(self) -> int:
        return self.w

    def coefficient(self, repair_id: int, src_id: int) -> int:
        rid, sid = repair_id & 0xFFFFFFFF, src_id & 0xFFFFFFFF
        if self.w == 8:
            return self._L.ntc_gf256_coefficient(rid, sid)
        return self._L.ntc_gf_coefficient(self.w, rid, sid)

    def multiply_size(self, size: int, coeff: int) -> int:
        if self.w == 8:
            return self._L.ntc_gf256_multiply_size(size, coeff)
        return self._L.ntc_gf_multiply_size(self.w, size, coeff & 0xFFFFFFFF)

    def multiply_scalar(self, x: int, y: int) -> int:
        if self.w == 8:
            return self._L.ntc_gf256_multiply(x, y)
        return self._L.ntc_gf_multiply(self.w, x & 0xFFFFFFFF, y & 0xFFFFFFFF)

    def invert(self, x: int) -> int:
        if x == 0:
            raise ZeroDivisionError(f"0 has no inverse in GF(2^{self.w})")
        if self.w == 8:
            return self._L.ntc_gf256_invert(x)
        return self._L.ntc_gf_invert(self.w, x & 0xFFFFFFFF)

    def _region(self, src: torch.Tensor, dst: torch.Tensor, length: int, coeff: int, add: int):
        if src.dtype != torch.uint8 or dst.dtype != torch.uint8:
            raise TypeError("regions are uint8 tensors")
        if not (src.is_cuda and dst.is_cuda) or src.device != dst.device:
            raise ValueError("regions must be device tensors on the same device")
        if length > src.numel() or length > dst.numel():
            raise ValueError("length exceeds region")
        eng = Engine.get(src.device)
        if self.w == 8:
            _native.check(self._L.ntc_gf256_region_multiply(
                eng.handle, src.data_ptr(), dst.data_ptr(), length, coeff & 0xFF, add,
                _stream(src.device)), "ntc_gf256_region_multiply")
        else:
            _native.check(self._L.ntc_gf_region_multiply(
                eng.handle, self.w, src.data_ptr(), dst.data_ptr(), length, coeff & 0xFFFFFFFF,
                add, _stream(src.device)), "ntc_gf_region_multiply")

    def multiply(self, src: torch.Tensor, dst: torch.Tensor, length: int, coeff: int):
        """dst[:length] = coeff * src[:length]  (galois_field.hh:65-75)."""
        self._region(src, dst, length, coeff, 0)

    def multiply_add(self, src: torch.Tensor, dst: torch.Tensor, length: int, coeff: int):
        """dst[:length] ^= coeff * src[:length]  (galois_field.hh:83-92)."""
        self._region(src, dst, length, coeff, 1)


def combine(w: int, inputs: torch.Tensor, coef: torch.Tensor, out: torch.Tensor | None = None):
    """Batched combination in GF(2^w): out[g][j] = sum_i coef[g][i][j] * inputs[g][i]
    (ntc_gf_combine_batch).  inputs [G, k, stride] uint8 (stride % 16 == 0), coef [G, k, rows]
    int32/uint32 field elements."""
    G, k, stride = inputs.shape
    rows = coef.shape[2]
    dev = inputs.device
    _require(inputs, "inputs", _U8, (G, k, stride), dev)
    _require(coef, "coef", _U32, (G, k, rows), dev)
    if out is None:
        out = torch.empty((G, rows, stride), dtype=torch.uint8, device=dev)
    eng = Engine.get(dev)
    _native.check(_native.load().ntc_gf_combine_batch(eng.handle, w, G, k, rows, stride,
                                                      inputs.data_ptr(), coef.data_ptr(),
                                                      out.data_ptr(), _stream(dev)),
                  "ntc_gf_combine_batch")
    return out


@dataclass
class EncodeResult:
    repairs: torch.Tensor      # [G, r, stride] uint8
    encoded_size: torch.Tensor  # [G, r] int16 (u16 bits)
    symbol_len: torch.Tensor   # [G] int16 (u16 bits): repair symbol length = max source length


class BatchEncoder:
    """G generations x (k sources -> r repairs), reference coefficient schedule."""

    def __init__(self, k: int, r: int, device: int | torch.device = 0, engine: Engine | None = None):
        # `engine`: a private Engine (own workspace) for launches that run concurrently with the
        # device's shared engine on other streams (HostPipeline); default the per-device one.
        self.k, self.r = int(k), int(r)
        self.engine = engine if engine is not None else Engine.get(device)
        self.device = self.engine.device

    def __call__(self, src: torch.Tensor, src_len: torch.Tensor, sid_base: torch.Tensor | None = None,
                 rid_base: torch.Tensor | None = None, out: EncodeResult | None = None) -> EncodeResult:
        G, k, stride = src.shape
        if k != self.k:
            raise ValueError(f"expected k={self.k}, got {k}")
        dev = self.device
        _require(src, "src", _U8, (G, k, stride), dev)
        _require(src_len, "src_len", _U16, (G, k), dev)
        if sid_base is not None:
            _require(sid_base, "sid_base", _U32, (G,), dev)
        if rid_base is not None:
            _require(rid_base, "rid_base", _U32, (G,), dev)
        if out is None:
            out = EncodeResult(torch.empty((G, self.r, stride), dtype=torch.uint8, device=dev),
                               torch.empty((G, self.r), dtype=torch.int16, device=dev),
                               torch.empty((G,), dtype=torch.int16, device=dev))
        L = _native.load()
        _native.check(L.ntc_gf256_encode_batch(self.engine.handle, G, k, self.r, stride,
                                               src.data_ptr(), src_len.data_ptr(), _ptr(sid_base),
                                               _ptr(rid_base), out.repairs.data_ptr(),
                                               out.encoded_size.data_ptr(),
                                               out.symbol_len.data_ptr(), _stream(dev)),
                      "ntc_gf256_encode_batch")
        return out


class BatchDecoder:
    """In-place generation decode; returns a [G, 12] uint8 status tensor (see STATUS_DTYPE)."""

    def __init__(self, k: int, r: int, device: int | torch.device = 0, engine: Engine | None = None):
        # `engine`: a private Engine (own workspace) for launches that run concurrently with the
        # device's shared engine on other streams (HostPipeline); default the per-device one.
        self.k, self.r = int(k), int(r)
        self.engine = engine if engine is not None else Engine.get(device)
        self.device = self.engine.device

    def __call__(self, src: torch.Tensor, src_len: torch.Tensor, src_mask: torch.Tensor,
                 rep: torch.Tensor, rep_size: torch.Tensor, rep_mask: torch.Tensor,
                 sid_base: torch.Tensor | None = None, rid_base: torch.Tensor | None = None,
                 status: torch.Tensor | None = None) -> torch.Tensor:
        G, k, stride = src.shape
        dev = self.device
        if k != self.k:
            raise ValueError(f"expected k={self.k}, got {k}")
        _require(src, "src", _U8, (G, k, stride), dev)
        _require(src_len, "src_len", _U16, (G, k), dev)
        _require(src_mask, "src_mask", _U8, (G, k), dev)
        _require(rep, "rep", _U8, (G, self.r, stride), dev)
        _require(rep_size, "rep_size", _U16, (G, self.r), dev)
        _require(rep_mask, "rep_mask", _U8, (G, self.r), dev)
        if sid_base is not None:
            _require(sid_base, "sid_base", _U32, (G,), dev)
        if rid_base is not None:
            _require(rid_base, "rid_base", _U32, (G,), dev)
        if status is None:
            status = torch.empty((G, STATUS_BYTES), dtype=torch.uint8, device=dev)
        L = _native.load()
        _native.check(L.ntc_gf256_decode_batch(self.engine.handle, G, k, self.r, stride,
                                               src.data_ptr(), src_len.data_ptr(),
                                               src_mask.data_ptr(), rep.data_ptr(),
                                               rep_size.data_ptr(), rep_mask.data_ptr(),
                                               _ptr(sid_base), _ptr(rid_base), status.data_ptr(),
                                               _stream(dev)),
                      "ntc_gf256_decode_batch")
        return status


# Per-packet outcome of Wire.read_packets (NTC_PKT_* in include/netcode/gpu.h).
PKT_SOURCE, PKT_REPAIR, PKT_ACK, PKT_BAD_TYPE, PKT_OVERFLOW, PKT_OUT_OF_BATCH, PKT_TOO_LARGE, \
    PKT_NOT_GENERATION = range(8)


@dataclass
class ReceivedBatch:
    """A batch layout filled from wire packets (the inputs of BatchDecoder)."""
    src: torch.Tensor        # [G, k, stride] uint8
    src_len: torch.Tensor    # [G, k] int16 (u16 bits)
    src_mask: torch.Tensor   # [G, k] uint8
    rep: torch.Tensor        # [G, r, stride] uint8
    rep_size: torch.Tensor   # [G, r] int16 (u16 bits): encoded sizes
    rep_mask: torch.Tensor   # [G, r] uint8
    status: torch.Tensor     # [npkts] uint8, PKT_*


class Wire:
    """netcode's packetizer (netcode/detail/packetizer.hh) over whole batches on the device.

    Packets live in fixed-size slots -- a [npkts, pkt_stride] uint8 tensor plus an [npkts] int32
    length tensor, the shape of a sendmmsg / recvmmsg batch:

    * :meth:`write_repairs` -- ``packetizer::write_repair`` (packetizer.hh:90-122) for every
      repair of an :class:`EncodeResult`;
    * :meth:`write_sources` -- ``packetizer::write_source`` (:165-183) for every source slot;
    * :meth:`read_packets` -- ``decoder::operator()(packet)`` dispatch + ``read_source`` /
      ``read_repair`` (:125-158, 186-218) into the :class:`BatchDecoder` layout;
    * :meth:`unpack_slots` / :meth:`pack_slots` -- packed rows of only the received (or only the
      lost) sources <-> the generation slots, so host-resident callers move just those bytes.
    """

    def __init__(self, device: int | torch.device = 0):
        self.engine = Engine.get(device)
        self.device = self.engine.device

    @staticmethod
    def repair_packet_bytes(k: int, stride: int) -> int:
        return int(_native.load().ntc_gf256_repair_packet_bytes(k, stride))

    @staticmethod
    def source_packet_bytes(stride: int) -> int:
        return (7 + stride + 15) // 16 * 16

    def _slots(self, n, pkt_stride):
        return (torch.empty((n, pkt_stride), dtype=torch.uint8, device=self.device),
                torch.empty((n,), dtype=torch.int32, device=self.device))

    def write_repairs(self, enc: EncodeResult, k: int, sid_base: torch.Tensor | None = None,
                      rid_base: torch.Tensor | None = None, pkt_stride: int | None = None):
        G, r, stride = enc.repairs.shape
        dev = self.device
        for t, n in ((sid_base, "sid_base"), (rid_base, "rid_base")):
            if t is not None:
                _require(t, n, _U32, (G,), dev)
        pkt_stride = pkt_stride or self.repair_packet_bytes(k, stride)
        pkts, lens = self._slots(G * r, pkt_stride)
        _native.check(_native.load().ntc_gf256_write_repairs(
            self.engine.handle, G, k, r, stride, enc.repairs.data_ptr(),
            enc.encoded_size.data_ptr(), enc.symbol_len.data_ptr(), _ptr(sid_base),
            _ptr(rid_base), pkts.data_ptr(), pkt_stride, lens.data_ptr(), _stream(dev)),
            "ntc_gf256_write_repairs")
        return pkts, lens

    def write_sources(self, src: torch.Tensor, src_len: torch.Tensor,
                      sid_base: torch.Tensor | None = None, pkt_stride: int | None = None):
        G, k, stride = src.shape
        dev = self.device
        _require(src, "src", _U8, (G, k, stride), dev)
        _require(src_len, "src_len", _U16, (G, k), dev)
        if sid_base is not None:
            _require(sid_base, "sid_base", _U32, (G,), dev)
        pkt_stride = pkt_stride or self.source_packet_bytes(stride)
        pkts, lens = self._slots(G * k, pkt_stride)
        _native.check(_native.load().ntc_gf256_write_sources(
            self.engine.handle, G, k, stride, src.data_ptr(), src_len.data_ptr(), _ptr(sid_base),
            pkts.data_ptr(), pkt_stride, lens.data_ptr(), _stream(dev)),
            "ntc_gf256_write_sources")
        return pkts, lens

    def read_packets(self, pkts: torch.Tensor, pkt_len: torch.Tensor, G: int, k: int, r: int,
                     stride: int, sid0: int = 0, rid0: int = 0,
                     out: ReceivedBatch | None = None, append: bool = False) -> ReceivedBatch:
        """append=True (ntc_gf256_read_packets_append): add to `out` what earlier calls stored
        instead of resetting its lengths / masks first (a second recvmmsg batch)."""
        n, pkt_stride = pkts.shape
        dev = self.device
        _require(pkts, "pkts", _U8, (n, pkt_stride), dev)
        _require(pkt_len, "pkt_len", _U32, (n,), dev)
        if out is None:
            out = ReceivedBatch(
                torch.empty((G, k, stride), dtype=torch.uint8, device=dev),
                torch.empty((G, k), dtype=torch.int16, device=dev),
                torch.empty((G, k), dtype=torch.uint8, device=dev),
                torch.empty((G, r, stride), dtype=torch.uint8, device=dev),
                torch.empty((G, r), dtype=torch.int16, device=dev),
                torch.empty((G, r), dtype=torch.uint8, device=dev),
                torch.empty((n,), dtype=torch.uint8, device=dev))
        if append and out is None:
            raise ValueError("append needs the batch of an earlier read_packets call")
        if out is not None and out.status.numel() < n:
            raise ValueError(f"out.status holds {out.status.numel()} packet outcomes, {n} packets given")
        L = _native.load()
        fn = L.ntc_gf256_read_packets_append if append else L.ntc_gf256_read_packets
        _native.check(fn(
            self.engine.handle, n, pkts.data_ptr(), pkt_stride, pkt_len.data_ptr(), G, k, r,
            stride, sid0 & 0xFFFFFFFF, rid0 & 0xFFFFFFFF, out.src.data_ptr(),
            out.src_len.data_ptr(), out.src_mask.data_ptr(), out.rep.data_ptr(),
            out.rep_size.data_ptr(), out.rep_mask.data_ptr(), out.status.data_ptr(),
            _stream(dev)), "ntc_gf256_read_packets")
        return out

    def _pack_args(self, slots, mask, row_base, packed, row0):
        G, k, stride = slots.shape
        dev = self.device
        _require(slots, "slots", _U8, (G, k, stride), dev)
        _require(mask, "mask", _U8, (G, k), dev)
        _require(row_base, "row_base", _U32, (G,), dev)
        if packed.dtype != torch.uint8 or packed.device != dev or packed.dim() != 2 or \
                packed.shape[1] != stride or not packed.is_contiguous():
            raise ValueError(f"packed must be a contiguous uint8 [rows, {stride}] tensor on {dev}")
        return G, k, stride, row0 & 0xFFFFFFFF

    def unpack_slots(self, packed: torch.Tensor, row_base: torch.Tensor, mask: torch.Tensor,
                     slots: torch.Tensor, want: int = 1, zero_rest: bool = True, row0: int = 0):
        """Packed rows -> the selected slots ((mask != 0) == want) of slots [G, k, stride]
        (ntc_gf256_unpack_slots); row_base [G] u32 = first packed row of each generation.
        The caller sizes `packed` to hold every selected row (not checked on the device)."""
        G, k, stride, row0 = self._pack_args(slots, mask, row_base, packed, row0)
        _native.check(_native.load().ntc_gf256_unpack_slots(
            self.engine.handle, G, k, stride, packed.data_ptr(), row_base.data_ptr(), row0,
            mask.data_ptr(), int(bool(want)), slots.data_ptr(), int(bool(zero_rest)),
            _stream(self.device)), "ntc_gf256_unpack_slots")
        return slots

    def pack_slots(self, slots: torch.Tensor, mask: torch.Tensor, row_base: torch.Tensor,
                   packed: torch.Tensor, want: int = 0, row0: int = 0):
        """Selected slots ((mask != 0) == want) of slots [G, k, stride] -> packed rows
        (ntc_gf256_pack_slots)."""
        G, k, stride, row0 = self._pack_args(slots, mask, row_base, packed, row0)
        _native.check(_native.load().ntc_gf256_pack_slots(
            self.engine.handle, G, k, stride, slots.data_ptr(), mask.data_ptr(),
            int(bool(want)), row_base.data_ptr(), row0, packed.data_ptr(),
            _stream(self.device)), "ntc_gf256_pack_slots")
        return packed


def status_to_numpy(status: torch.Tensor) -> np.ndarray:
    """[G, 12] uint8 device tensor -> structured numpy array (STATUS_DTYPE)."""
    return status.cpu().numpy().view(STATUS_DTYPE).reshape(-1)


class DenseCode:
    """Dense (non-reference) GF(2^8) codes, BASELINE config 5: caller-chosen coefficient matrices,
    device Gauss-Jordan inversion (the work of detail::invert, invert_matrix.cc:9-128) and the
    region MAC of attempt_full_decoding (detail/decoder.cc:503-534) for n up to 1024."""

    def __init__(self, device: int | torch.device = 0):
        self.engine = Engine.get(device)
        self.device = self.engine.device

    def encode(self, mat: torch.Tensor, src: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """rep[g][j] = sum_i mat[g][j][i] * src[g][i];  mat [G, r, k], src [G, k, stride]."""
        G, k, stride = src.shape
        r = mat.shape[1]
        dev = self.device
        _require(mat, "mat", _U8, (G, r, k), dev)
        _require(src, "src", _U8, (G, k, stride), dev)
        if out is None:
            out = torch.empty((G, r, stride), dtype=torch.uint8, device=dev)
        _require(out, "out", _U8, (G, r, stride), dev)
        L = _native.load()
        _native.check(L.ntc_gf256_dense_encode_batch(self.engine.handle, G, k, r, stride,
                                                     mat.data_ptr(), src.data_ptr(),
                                                     out.data_ptr(), _stream(dev)),
                      "ntc_gf256_dense_encode_batch")
        return out

    def decode(self, mat: torch.Tensor, rep: torch.Tensor, out: torch.Tensor | None = None,
               ok: torch.Tensor | None = None):
        """(out, ok): out[g] = mat[g]^-1 rep[g];  ok[g] = 0 marks a singular matrix."""
        G, n, stride = rep.shape
        dev = self.device
        _require(mat, "mat", _U8, (G, n, n), dev)
        _require(rep, "rep", _U8, (G, n, stride), dev)
        if out is None:
            out = torch.empty((G, n, stride), dtype=torch.uint8, device=dev)
        if ok is None:
            ok = torch.empty((G,), dtype=torch.uint8, device=dev)
        _require(out, "out", _U8, (G, n, stride), dev)
        _require(ok, "ok", _U8, (G,), dev)
        L = _native.load()
        _native.check(L.ntc_gf256_dense_decode_batch(self.engine.handle, G, n, stride,
                                                     mat.data_ptr(), rep.data_ptr(),
                                                     out.data_ptr(), ok.data_ptr(), _stream(dev)),
                      "ntc_gf256_dense_decode_batch")
        return out, ok

    def invert(self, mat: torch.Tensor):
        """(inv, ok) for G n x n matrices."""
        G, n, _ = mat.shape
        dev = self.device
        _require(mat, "mat", _U8, (G, n, n), dev)
        inv = torch.empty((G, n, n), dtype=torch.uint8, device=dev)
        ok = torch.empty((G,), dtype=torch.uint8, device=dev)
        L = _native.load()
        _native.check(L.ntc_gf256_dense_invert_batch(self.engine.handle, G, n, mat.data_ptr(),
                                                     inv.data_ptr(), ok.data_ptr(), _stream(dev)),
                      "ntc_gf256_dense_invert_batch")
        return inv, ok
