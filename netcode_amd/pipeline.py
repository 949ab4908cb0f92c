"""Host-resident batch coding: generations that start and end in pinned host memory (the
reference's UDP socket buffers, `examples/` of ahamez/netcode) stream through the device in
chunks, so the PCIe copies of one chunk overlap the kernels and the opposite-direction copies of
the others.

Each of `depth` slots owns a HIP stream, a private Engine (its own coefficient / plan / jump-offset
workspace, so launches on different streams never share scratch) and device buffers for one chunk.
Chunk c runs on slot c % depth: H2D -> encode/decode kernels -> D2H, all in stream order, so a
slot's buffers are reused only after its previous chunk's D2H has been issued behind them.
Results are byte-identical to one device-resident call over the whole batch (tests/
test_gpu_pipeline.py): generations are independent and every chunk keeps its generations' id
bases -- with no explicit bases, chunk generations g0..g1 get the whole-batch defaults g*k / g*r
(u32 wraparound), exactly what one BatchEncoder call over all G generations uses.
"""
from __future__ import annotations

import numpy as np
import torch

from .engine import BatchDecoder, BatchEncoder, Engine, EncodeResult, STATUS_BYTES

_I16 = (torch.int16, torch.uint16)


def _pinned(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cpu" or not t.is_pinned():
        raise ValueError(f"{name} must be a pinned host tensor (torch.Tensor.pin_memory())")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def _default_bases(g0: int, g1: int, per_gen: int, device) -> torch.Tensor:
    """u32 id bases (g * per_gen) mod 2^32 for generations g0..g1-1, as an int32 device tensor
    (the kernels' fallback when no base pointer is given is the same product in u32)."""
    v = (torch.arange(g0, g1, dtype=torch.int64) * per_gen) & 0xFFFFFFFF
    v = torch.where(v >= 2**31, v - 2**32, v)
    return v.to(torch.int32).to(device, non_blocking=False)


class HostPipeline:
    """Chunked, stream-overlapped encode / decode of host-resident generation batches."""

    def __init__(self, k: int, r: int, stride: int, chunk: int, device: int | torch.device = 0,
                 depth: int = 3):
        if chunk <= 0 or depth <= 0:
            raise ValueError("chunk and depth must be positive")
        self.k, self.r, self.stride, self.chunk, self.depth = int(k), int(r), int(stride), int(chunk), int(depth)
        dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.device = dev
        self.streams = [torch.cuda.Stream(dev) for _ in range(depth)]
        self.engines = [Engine(dev) for _ in range(depth)]
        for e in self.engines:
            e.reserve(chunk, k, r)
        self.enc = [BatchEncoder(k, r, dev, engine=e) for e in self.engines]
        self.dec = [BatchDecoder(k, r, dev, engine=e) for e in self.engines]
        u8, i16 = torch.uint8, torch.int16
        C = chunk
        self.d_src = [torch.empty((C, k, stride), dtype=u8, device=dev) for _ in range(depth)]
        self.d_len = [torch.empty((C, k), dtype=i16, device=dev) for _ in range(depth)]
        self.d_mask = [torch.empty((C, k), dtype=u8, device=dev) for _ in range(depth)]
        self.d_rmask = [torch.empty((C, r), dtype=u8, device=dev) for _ in range(depth)]
        self.d_out = [EncodeResult(torch.empty((C, r, stride), dtype=u8, device=dev),
                                   torch.empty((C, r), dtype=i16, device=dev),
                                   torch.empty((C,), dtype=i16, device=dev)) for _ in range(depth)]
        self.d_status = [torch.empty((C, STATUS_BYTES), dtype=u8, device=dev) for _ in range(depth)]

    def _chunks(self, G: int):
        for c, g0 in enumerate(range(0, G, self.chunk)):
            yield c % self.depth, g0, min(G, g0 + self.chunk)

    # expected (dtypes, trailing shape) of every host argument, by name
    def _spec(self, name: str):
        k, r, S = self.k, self.r, self.stride
        u8 = (torch.uint8,)
        return {"h_src": (u8, (k, S)), "h_rx": (u8, (k, S)), "h_rep": (u8, (r, S)),
                "h_src_len": (_I16, (k,)), "h_rx_len": (_I16, (k,)), "h_rep_size": (_I16, (r,)),
                "h_rep_len": (_I16, ()), "h_mask": (u8, (k,)), "h_rmask": (u8, (r,)),
                "h_status": (u8, (STATUS_BYTES,))}[name]

    def _check(self, G: int, **tensors):
        """Every host tensor: pinned, contiguous, [G, ...] with this pipeline's k / r / stride and
        the dtype the device side expects (copy_ would silently cast or broadcast otherwise)."""
        for name, t in tensors.items():
            if t is None:
                continue
            _pinned(t, name)
            dtypes, tail = self._spec(name)
            if t.dtype not in dtypes:
                raise TypeError(f"{name} must have dtype {dtypes}, got {t.dtype}")
            if tuple(t.shape) != (G,) + tail:
                raise ValueError(f"{name} must have shape {(G,) + tail}, got {tuple(t.shape)}")

    def _check_bases(self, G: int, **bases):
        for name, t in bases.items():
            if t is None:
                continue
            if t.device != self.device or t.dtype not in (torch.int32, torch.uint32) or \
                    tuple(t.shape) != (G,) or not t.is_contiguous():
                raise ValueError(f"{name} must be a contiguous int32/uint32 [{G}] tensor on {self.device}")

    def _bases(self, G: int, sid_base, rid_base):
        """Explicit bases, or the whole-batch defaults (built on the caller's current stream,
        which every chunk stream waits for in _fork)."""
        self._check_bases(G, sid_base=sid_base, rid_base=rid_base)
        if sid_base is None:
            sid_base = _default_bases(0, G, self.k, self.device)
        if rid_base is None:
            rid_base = _default_bases(0, G, self.r, self.device)
        return sid_base, rid_base

    def _fork(self):
        # work the caller queued before this call (device id bases, earlier copies) comes first
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(cur)

    def _join(self):
        cur = torch.cuda.current_stream(self.device)
        for s in self.streams:
            cur.wait_stream(s)

    def encode(self, h_src, h_src_len, h_rep, h_rep_size, sid_base=None, rid_base=None,
               h_rep_len=None):
        """h_src [G,k,stride] u8, h_src_len [G,k] i16 -> h_rep [G,r,stride] u8, h_rep_size [G,r]
        i16, optionally h_rep_len [G] i16 (repair symbol length = max source length, what a repair
        packet's header carries) -- pinned host tensors.  sid_base / rid_base: optional device u32
        [G] id bases.  Asynchronous with respect to the host; the caller's current stream waits
        for all chunks."""
        G = h_src.shape[0]
        self._check(G, h_src=h_src, h_src_len=h_src_len, h_rep=h_rep, h_rep_size=h_rep_size,
                    h_rep_len=h_rep_len)
        sid_base, rid_base = self._bases(G, sid_base, rid_base)
        self._fork()
        for s, g0, g1 in self._chunks(G):
            n = g1 - g0
            with torch.cuda.stream(self.streams[s]):
                src, ln, out = self.d_src[s][:n], self.d_len[s][:n], self.d_out[s]
                src.copy_(h_src[g0:g1], non_blocking=True)
                ln.copy_(h_src_len[g0:g1], non_blocking=True)
                o = EncodeResult(out.repairs[:n], out.encoded_size[:n], out.symbol_len[:n])
                self.enc[s](src, ln, sid_base[g0:g1], rid_base[g0:g1], o)
                h_rep[g0:g1].copy_(o.repairs, non_blocking=True)
                h_rep_size[g0:g1].copy_(o.encoded_size, non_blocking=True)
                if h_rep_len is not None:
                    h_rep_len[g0:g1].copy_(o.symbol_len, non_blocking=True)
        self._join()

    def decode(self, h_rx, h_rx_len, h_mask, h_rep, h_rep_size, h_rmask, h_status,
               sid_base=None, rid_base=None):
        """In-place decode of host-resident generations: received sources h_rx [G,k,stride]
        (lost slots are overwritten with the recovered sources, and their h_rx_len entries with
        the decoded sizes), h_rx_len / h_mask [G,k], repairs h_rep [G,r,stride] / h_rep_size /
        h_rmask [G,r], status out h_status [G,12] u8."""
        G = h_rx.shape[0]
        self._check(G, h_rx=h_rx, h_rx_len=h_rx_len, h_mask=h_mask, h_rep=h_rep,
                    h_rep_size=h_rep_size, h_rmask=h_rmask, h_status=h_status)
        sid_base, rid_base = self._bases(G, sid_base, rid_base)
        self._fork()
        for s, g0, g1 in self._chunks(G):
            n = g1 - g0
            with torch.cuda.stream(self.streams[s]):
                rx, ln, mk = self.d_src[s][:n], self.d_len[s][:n], self.d_mask[s][:n]
                rep, rsz, rmk = self.d_out[s].repairs[:n], self.d_out[s].encoded_size[:n], self.d_rmask[s][:n]
                st = self.d_status[s][:n]
                for d, h in ((rx, h_rx), (ln, h_rx_len), (mk, h_mask), (rep, h_rep), (rsz, h_rep_size),
                             (rmk, h_rmask)):
                    d.copy_(h[g0:g1], non_blocking=True)
                self.dec[s](rx, ln, mk, rep, rsz, rmk, sid_base[g0:g1], rid_base[g0:g1], st)
                h_rx[g0:g1].copy_(rx, non_blocking=True)
                h_rx_len[g0:g1].copy_(ln, non_blocking=True)
                h_status[g0:g1].copy_(st, non_blocking=True)
        self._join()

    @staticmethod
    def row_bases(h_mask: torch.Tensor):
        """(rx_base, lost_base, n_rx, n_lost) for a host mask [G, k]: the first packed row of each
        generation among the received (mask != 0) and the lost slots, as int32 [G] host tensors."""
        rx = (h_mask != 0).sum(1, dtype=torch.int64)
        lost = h_mask.shape[1] - rx
        rx_base = torch.cumsum(rx, 0) - rx
        lost_base = torch.cumsum(lost, 0) - lost
        return (rx_base.to(torch.int32), lost_base.to(torch.int32), int(rx.sum()), int(lost.sum()))

    def encode_decode_packed(self, h_src, h_src_len, h_rep, h_rep_size, h_rx_packed, h_rx_len,
                             h_mask, h_rmask, h_rec_packed, h_status, sid_base=None,
                             rid_base=None):
        """Loopback of one batch moving only the bytes a real sender / receiver pair moves: the
        sources H2D for the encoder, the repairs D2H; then only the RECEIVED sources H2D, packed
        (h_rx_packed [n_rx, stride], generation-major, slot order within a generation, as
        :meth:`row_bases` numbers them), and only the LOST slots D2H, packed (h_rec_packed
        [n_lost, stride]: the recovered sources, zeros where a generation did not decode --
        h_status says which).  h_rx_len [G, k] goes in with the received lengths and comes back
        with the decoded sizes in the lost slots.  Per chunk, the received rows are unpacked into
        the generation slots on the device (lost slots zeroed), decoded, and the lost slots packed
        again (ntc_gf256_unpack_slots / ntc_gf256_pack_slots).  Same bytes as encode_decode()."""
        from .engine import Wire
        G = h_src.shape[0]
        self._check(G, h_src=h_src, h_src_len=h_src_len, h_rep=h_rep, h_rep_size=h_rep_size,
                    h_rx_len=h_rx_len, h_mask=h_mask, h_rmask=h_rmask, h_status=h_status)
        rx_base, lost_base, n_rx, n_lost = self.row_bases(h_mask)
        for name, t, n in (("h_rx_packed", h_rx_packed, n_rx), ("h_rec_packed", h_rec_packed, n_lost)):
            _pinned(t, name)
            if t.dtype != torch.uint8 or tuple(t.shape) != (n, self.stride):
                raise ValueError(f"{name} must be uint8 [{n}, {self.stride}], got {t.dtype} {tuple(t.shape)}")
        sid_base, rid_base = self._bases(G, sid_base, rid_base)
        wire = Wire(self.device)
        if not hasattr(self, "d_rows"):
            self.d_rows = [torch.empty((self.chunk * self.k, self.stride), dtype=torch.uint8,
                                       device=self.device) for _ in range(self.depth)]
        d_rx_base = rx_base.to(self.device)
        d_lost_base = lost_base.to(self.device)
        self._fork()
        for s, g0, g1 in self._chunks(G):
            n = g1 - g0
            r0, r1 = int(rx_base[g0]), (int(rx_base[g1]) if g1 < G else n_rx)
            l0, l1 = int(lost_base[g0]), (int(lost_base[g1]) if g1 < G else n_lost)
            with torch.cuda.stream(self.streams[s]):
                buf, ln, mk, rmk = self.d_src[s][:n], self.d_len[s][:n], self.d_mask[s][:n], self.d_rmask[s][:n]
                out, st, rows = self.d_out[s], self.d_status[s][:n], self.d_rows[s]
                o = EncodeResult(out.repairs[:n], out.encoded_size[:n], out.symbol_len[:n])
                sid, rid = sid_base[g0:g1], rid_base[g0:g1]
                buf.copy_(h_src[g0:g1], non_blocking=True)
                ln.copy_(h_src_len[g0:g1], non_blocking=True)
                self.enc[s](buf, ln, sid, rid, o)
                h_rep[g0:g1].copy_(o.repairs, non_blocking=True)
                h_rep_size[g0:g1].copy_(o.encoded_size, non_blocking=True)
                for d, h in ((ln, h_rx_len), (mk, h_mask), (rmk, h_rmask)):
                    d.copy_(h[g0:g1], non_blocking=True)
                rows[:r1 - r0].copy_(h_rx_packed[r0:r1], non_blocking=True)
                # the decoder's slots reuse the source buffer (stream order: the encode has read it)
                wire.unpack_slots(rows[:max(r1 - r0, 1)], d_rx_base[g0:g1], mk, buf, want=1,
                                  zero_rest=True, row0=r0)
                self.dec[s](buf, ln, mk, o.repairs, o.encoded_size, rmk, sid, rid, st)
                if l1 > l0:
                    wire.pack_slots(buf, mk, d_lost_base[g0:g1], rows[:l1 - l0], want=0, row0=l0)
                    h_rec_packed[l0:l1].copy_(rows[:l1 - l0], non_blocking=True)
                h_rx_len[g0:g1].copy_(ln, non_blocking=True)
                h_status[g0:g1].copy_(st, non_blocking=True)
        self._join()

    def encode_decode_wire(self, h_src, h_src_len, h_rep_pkts, h_rep_pkt_len, h_rx_pkts, h_rx_pkt_len,
                           rx_first, h_mask, h_rec_packed, h_dec_len, h_status, sid_host, rid_host,
                           sid_base, rid_base):
        """Loopback of one batch through the WIRE format, socket buffer to socket buffer (the path of
        the reference's examples: the sender hands payloads in and takes packets out; the receiver
        hands packets in and takes recovered payloads out).  Per chunk of generations:

        * sender: sources H2D -> encode -> ``write_repairs`` (packetizer.hh:90-122) -> the repair
          packets D2H into h_rep_pkts [G*r, rps] / h_rep_pkt_len [G*r] (a sendmmsg batch; the source
          packets are the caller's payloads behind a 7-byte header);
        * receiver: its received packets H2D -- the source packets h_rx_pkts [N, sps] /
          h_rx_pkt_len [N] (generations g0..g1 own rows rx_first[g0]..rx_first[g1]) and the repair
          packets the sender put in h_rep_pkts -- -> ``read_packets`` + ``read_packets_append``
          (decoder.hh dispatch + read_source / read_repair) into its own slots -> decode -> the
          LOST slots packed (``pack_slots``) and D2H into h_rec_packed [n_lost, stride], the
          decoded sizes into h_dec_len [G, k], the status into h_status.

        sid_host / rid_host: the u32 id bases as host sequences (read_packets maps ids to slots
        from the chunk's first bases); sid_base / rid_base the same on the device.  The lost rows'
        offsets come from h_mask, the loss pattern the caller applied."""
        from .engine import ReceivedBatch, Wire
        G = h_src.shape[0]
        k, r, stride = self.k, self.r, self.stride
        self._check(G, h_src=h_src, h_src_len=h_src_len, h_mask=h_mask, h_status=h_status)
        self._check_bases(G, sid_base=sid_base, rid_base=rid_base)
        rps = Wire.repair_packet_bytes(k, stride)
        for name, t, shape, dt in (("h_rep_pkts", h_rep_pkts, (G * r, rps), torch.uint8),
                                   ("h_rep_pkt_len", h_rep_pkt_len, (G * r,), torch.int32),
                                   ("h_rx_pkt_len", h_rx_pkt_len, (h_rx_pkts.shape[0],), torch.int32),
                                   ("h_dec_len", h_dec_len, (G, k), torch.int16)):
            _pinned(t, name)
            if t.dtype != dt or tuple(t.shape) != shape:
                raise ValueError(f"{name} must be {dt} {shape}, got {t.dtype} {tuple(t.shape)}")
        _pinned(h_rx_pkts, "h_rx_pkts")
        sps = h_rx_pkts.shape[1]
        # read_packets maps a packet to generation (id - chunk's first base) // k (// r for repairs),
        # so within every chunk the bases must be contiguous: sid[g] = sid[g0] + (g - g0)*k (mod 2^32)
        sh = np.asarray(sid_host, dtype=np.uint64) & 0xFFFFFFFF
        rh = np.asarray(rid_host, dtype=np.uint64) & 0xFFFFFFFF
        if sh.shape != (G,) or rh.shape != (G,):
            raise ValueError(f"sid_host / rid_host must hold {G} id bases")
        for _, g0, g1 in self._chunks(G):
            off = np.arange(g1 - g0, dtype=np.uint64)
            if (((sh[g0:g1] - sh[g0] - off * k) & 0xFFFFFFFF) != 0).any() or \
               (((rh[g0:g1] - rh[g0] - off * r) & 0xFFFFFFFF) != 0).any():
                raise ValueError("encode_decode_wire needs contiguous id bases within each chunk "
                                 f"(generations {g0}..{g1 - 1}): sid[g] = sid[g0] + (g-g0)*k, "
                                 "rid[g] = rid[g0] + (g-g0)*r (mod 2^32)")
        _, lost_base, _, n_lost = self.row_bases(h_mask)
        wire = Wire(self.device)
        dev = self.device
        if not hasattr(self, "d_rows"):
            self.d_rows = [torch.empty((self.chunk * k, stride), dtype=torch.uint8, device=dev)
                           for _ in range(self.depth)]
        if getattr(self, "_wire_cap", None) != (rps, sps):
            C, D = self.chunk, self.depth
            self.d_rep_pkts = [torch.empty((C * r, rps), dtype=torch.uint8, device=dev) for _ in range(D)]
            self.d_rep_pkt_len = [torch.empty((C * r,), dtype=torch.int32, device=dev) for _ in range(D)]
            self.d_rx_rep_pkts = [torch.empty((C * r, rps), dtype=torch.uint8, device=dev) for _ in range(D)]
            self.d_rx_rep_len = [torch.empty((C * r,), dtype=torch.int32, device=dev) for _ in range(D)]
            self.d_rx_pkts = [torch.empty((C * k, sps), dtype=torch.uint8, device=dev) for _ in range(D)]
            self.d_rx_pkt_len = [torch.empty((C * k,), dtype=torch.int32, device=dev) for _ in range(D)]
            self.d_pkt_status = [torch.empty((C * (k + r),), dtype=torch.uint8, device=dev) for _ in range(D)]
            # the receiver's own slots: nothing of the sender's buffers is visible to it
            self.d_rxs = [torch.empty((C, k, stride), dtype=torch.uint8, device=dev) for _ in range(D)]
            self.d_rxrep = [torch.empty((C, r, stride), dtype=torch.uint8, device=dev) for _ in range(D)]
            self.d_rxrsz = [torch.empty((C, r), dtype=torch.int16, device=dev) for _ in range(D)]
            self._wire_cap = (rps, sps)
        d_lost_base = lost_base.to(dev)
        self._fork()
        for s, g0, g1 in self._chunks(G):
            n = g1 - g0
            p0, p1 = int(rx_first[g0]), int(rx_first[g1])
            l0, l1 = int(lost_base[g0]), (int(lost_base[g1]) if g1 < G else n_lost)
            with torch.cuda.stream(self.streams[s]):
                buf, ln, mk, rmk = self.d_src[s][:n], self.d_len[s][:n], self.d_mask[s][:n], self.d_rmask[s][:n]
                out, st, rows = self.d_out[s], self.d_status[s][:n], self.d_rows[s]
                o = EncodeResult(out.repairs[:n], out.encoded_size[:n], out.symbol_len[:n])
                sid, rid = sid_base[g0:g1], rid_base[g0:g1]
                # sender
                buf.copy_(h_src[g0:g1], non_blocking=True)
                ln.copy_(h_src_len[g0:g1], non_blocking=True)
                self.enc[s](buf, ln, sid, rid, o)
                rp, rl = self.d_rep_pkts[s][:n * r], self.d_rep_pkt_len[s][:n * r]
                _native_write_repairs(wire, o, k, sid, rid, rp, rl)
                h_rep_pkts[g0 * r:g1 * r].copy_(rp, non_blocking=True)
                h_rep_pkt_len[g0 * r:g1 * r].copy_(rl, non_blocking=True)
                # receiver: source packets, then the repair packets back from the sender's host
                # buffer (stream order: after their D2H), into slots of its own
                xp, xl = self.d_rx_pkts[s][:p1 - p0], self.d_rx_pkt_len[s][:p1 - p0]
                xp.copy_(h_rx_pkts[p0:p1], non_blocking=True)
                xl.copy_(h_rx_pkt_len[p0:p1], non_blocking=True)
                yp, yl = self.d_rx_rep_pkts[s][:n * r], self.d_rx_rep_len[s][:n * r]
                yp.copy_(h_rep_pkts[g0 * r:g1 * r], non_blocking=True)
                yl.copy_(h_rep_pkt_len[g0 * r:g1 * r], non_blocking=True)
                rx, rrep, rrsz = self.d_rxs[s][:n], self.d_rxrep[s][:n], self.d_rxrsz[s][:n]
                rb = ReceivedBatch(rx, ln, mk, rrep, rrsz, rmk, self.d_pkt_status[s][:p1 - p0])
                wire.read_packets(xp, xl, n, k, r, stride, int(sid_host[g0]), int(rid_host[g0]), out=rb)
                rb.status = self.d_pkt_status[s][p1 - p0:p1 - p0 + n * r]
                wire.read_packets(yp, yl, n, k, r, stride, int(sid_host[g0]), int(rid_host[g0]), out=rb,
                                  append=True)
                self.dec[s](rx, ln, mk, rrep, rrsz, rmk, sid, rid, st)
                if l1 > l0:
                    wire.pack_slots(rx, mk, d_lost_base[g0:g1], rows[:l1 - l0], want=0, row0=l0)
                    h_rec_packed[l0:l1].copy_(rows[:l1 - l0], non_blocking=True)
                h_dec_len[g0:g1].copy_(ln, non_blocking=True)
                h_status[g0:g1].copy_(st, non_blocking=True)
        self._join()

    def encode_decode(self, h_src, h_src_len, h_rep, h_rep_size, h_rx, h_rx_len, h_mask, h_rmask,
                      h_status, sid_base=None, rid_base=None):
        """Loopback of one batch (bench.py's host-resident rate): per chunk, sources H2D -> encode
        -> repairs D2H to h_rep, then received sources H2D -> decode with the chunk's repairs
        still on the device -> recovered sources, their decoded sizes and status D2H.  Same
        results as encode() then decode() with h_rep as the decoder's repairs."""
        G = h_src.shape[0]
        self._check(G, h_src=h_src, h_src_len=h_src_len, h_rep=h_rep, h_rep_size=h_rep_size,
                    h_rx=h_rx, h_rx_len=h_rx_len, h_mask=h_mask, h_rmask=h_rmask, h_status=h_status)
        sid_base, rid_base = self._bases(G, sid_base, rid_base)
        self._fork()
        for s, g0, g1 in self._chunks(G):
            n = g1 - g0
            with torch.cuda.stream(self.streams[s]):
                buf, ln, mk, rmk = self.d_src[s][:n], self.d_len[s][:n], self.d_mask[s][:n], self.d_rmask[s][:n]
                out, st = self.d_out[s], self.d_status[s][:n]
                o = EncodeResult(out.repairs[:n], out.encoded_size[:n], out.symbol_len[:n])
                sid, rid = sid_base[g0:g1], rid_base[g0:g1]
                buf.copy_(h_src[g0:g1], non_blocking=True)
                ln.copy_(h_src_len[g0:g1], non_blocking=True)
                self.enc[s](buf, ln, sid, rid, o)
                h_rep[g0:g1].copy_(o.repairs, non_blocking=True)
                h_rep_size[g0:g1].copy_(o.encoded_size, non_blocking=True)
                # the decoder's slots reuse the source buffer (stream order: the encode has read it)
                for d, h in ((buf, h_rx), (ln, h_rx_len), (mk, h_mask), (rmk, h_rmask)):
                    d.copy_(h[g0:g1], non_blocking=True)
                self.dec[s](buf, ln, mk, o.repairs, o.encoded_size, rmk, sid, rid, st)
                h_rx[g0:g1].copy_(buf, non_blocking=True)
                h_rx_len[g0:g1].copy_(ln, non_blocking=True)
                h_status[g0:g1].copy_(st, non_blocking=True)
        self._join()


def _native_write_repairs(wire, enc, k, sid, rid, pkts, lens):
    """ntc_gf256_write_repairs into caller-owned packet slots (Wire.write_repairs allocates)."""
    from . import _native
    from .engine import _ptr, _stream
    G, r, stride = enc.repairs.shape
    _native.check(_native.load().ntc_gf256_write_repairs(
        wire.engine.handle, G, k, r, stride, enc.repairs.data_ptr(), enc.encoded_size.data_ptr(),
        enc.symbol_len.data_ptr(), _ptr(sid), _ptr(rid), pkts.data_ptr(), pkts.shape[1],
        lens.data_ptr(), _stream(wire.device)), "ntc_gf256_write_repairs")
