// ntc_wire.hip -- netcode's wire format on the device.
//
// The reference serialises every packet through a byte-at-a-time handler on the host
// (netcode/detail/packetizer.hh: write_repair :90-122, write_source :165-183, read_repair :125-158,
// read_source :186-218; integers big-endian) and parses them back the same way.  Batched here:
//
//   ntc_gf256_write_repairs  one wire packet per repair of an encoded batch, into fixed-size slots
//                            of a device (or pinned, device-mapped) buffer, ready for sendmmsg;
//   ntc_gf256_write_sources  one wire packet per source slot;
//   ntc_gf256_read_packets   a batch of received wire packets (slot buffer + lengths, e.g. from
//                            recvmmsg) parsed and scattered into the generation layout the batched
//                            decoder consumes (slots zero-padded to the stride, masks, lengths,
//                            encoded sizes), with a per-packet status.
//
// All three are HBM-bound byte movers: one workgroup per packet, 16-byte stores per lane, the
// payload realigned from its 7-byte-offset position in the packet with v_alignbyte on aligned
// 16-byte loads (no byte loads on the payload path).  Header, id list and trailer bytes (a few
// dozen per packet) go through a per-byte path.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "engine.hh"
#include "netcode/gpu.h"

namespace ntcgpu {
namespace {

constexpr uint32_t kWireThreads = 256;

// 16 bytes starting `sh` bytes (wave-uniform, 0..15) past the 16-byte-aligned address p.  The
// second aligned block is read only when sh != 0 and only if it lies before `limit` (exclusive end
// of readable memory, relative to p); bytes past `limit` read as zero.
__device__ __forceinline__ uint4 load16_shifted(const uint8_t* p, uint32_t sh, uint32_t limit)
{
  const uint4 q0 = *reinterpret_cast<const uint4*>(p);
  if (sh == 0) return q0;
  const uint4 q1 = limit > 16u ? *reinterpret_cast<const uint4*>(p + 16) : make_uint4(0, 0, 0, 0);
  const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  const uint32_t b = sh & 3u;
  uint32_t d[5];
  switch (sh >> 2) {                     // uniform branch: which dword starts the window
    case 0: d[0] = w[0]; d[1] = w[1]; d[2] = w[2]; d[3] = w[3]; d[4] = w[4]; break;
    case 1: d[0] = w[1]; d[1] = w[2]; d[2] = w[3]; d[3] = w[4]; d[4] = w[5]; break;
    case 2: d[0] = w[2]; d[1] = w[3]; d[2] = w[4]; d[3] = w[5]; d[4] = w[6]; break;
    default: d[0] = w[3]; d[1] = w[4]; d[2] = w[5]; d[3] = w[6]; d[4] = w[7]; break;
  }
  // alignbyte(hi, lo, b) = ({hi, lo} >> 8b)[31:0]
  return make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], b), __builtin_amdgcn_alignbyte(d[2], d[1], b),
                    __builtin_amdgcn_alignbyte(d[3], d[2], b), __builtin_amdgcn_alignbyte(d[4], d[3], b));
}

// 16 bytes of a slot starting at (possibly negative) byte offset off; bytes outside [0, stride)
// read as zero.  Two guarded aligned loads, realigned like load16_shifted.
__device__ __forceinline__ uint4 slot16(const uint8_t* base, int32_t off, uint32_t stride)
{
  const int32_t a0 = off & ~15;                        // floor to 16 (two's complement)
  const uint32_t sh = static_cast<uint32_t>(off - a0);
  const uint4 z = make_uint4(0, 0, 0, 0);
  const uint4 q0 = (a0 >= 0 && static_cast<uint32_t>(a0) < stride)
                       ? *reinterpret_cast<const uint4*>(base + a0) : z;
  const uint4 q1 = (sh != 0 && a0 + 16 >= 0 && static_cast<uint32_t>(a0 + 16) < stride)
                       ? *reinterpret_cast<const uint4*>(base + a0 + 16) : z;
  if (sh == 0) return q0;
  const uint32_t w[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  const uint32_t b = sh & 3u;
  uint32_t d[5];
  switch (sh >> 2) {
    case 0: d[0] = w[0]; d[1] = w[1]; d[2] = w[2]; d[3] = w[3]; d[4] = w[4]; break;
    case 1: d[0] = w[1]; d[1] = w[2]; d[2] = w[3]; d[3] = w[4]; d[4] = w[5]; break;
    case 2: d[0] = w[2]; d[1] = w[3]; d[2] = w[4]; d[3] = w[5]; d[4] = w[6]; break;
    default: d[0] = w[3]; d[1] = w[4]; d[2] = w[5]; d[3] = w[6]; d[4] = w[7]; break;
  }
  return make_uint4(__builtin_amdgcn_alignbyte(d[1], d[0], b), __builtin_amdgcn_alignbyte(d[2], d[1], b),
                    __builtin_amdgcn_alignbyte(d[3], d[2], b), __builtin_amdgcn_alignbyte(d[4], d[3], b));
}

__device__ __forceinline__ uint32_t get_byte(const uint4& v, uint32_t i)
{
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
  return (w[i >> 2] >> (8u * (i & 3u))) & 0xFFu;
}

__device__ __forceinline__ void put_byte(uint4& v, uint32_t i, uint32_t b)
{
  uint32_t* w = reinterpret_cast<uint32_t*>(&v);
  const uint32_t sh = 8u * (i & 3u);
  w[i >> 2] = (w[i >> 2] & ~(0xFFu << sh)) | (b << sh);
}

// ---- serialisation --------------------------------------------------------------------------

// Source-id list of a whole generation (sidb .. sidb+k-1) in the packetizer's run-length form
// (packetizer.hh:263-309): u16 count = 1 + runs, u32 first id, then per run u8 length and u16
// delta (= 1); consecutive equal deltas are grouped in runs of at most 255.
__device__ __forceinline__ uint32_t ids_bytes(uint32_t k)
{
  return k == 0 ? 2u : 6u + 3u * ((k - 1u + 254u) / 255u);
}

__device__ __forceinline__ uint32_t ids_byte(uint32_t k, uint32_t sidb, uint32_t q)
{
  const uint32_t nruns = k == 0 ? 0u : (k - 1u + 254u) / 255u;
  const uint32_t count = k == 0 ? 0u : 1u + nruns;
  if (q < 2) return (count >> (8 * (1 - q))) & 0xFFu;
  if (q < 6) return (sidb >> (8 * (5 - q))) & 0xFFu;
  const uint32_t run = (q - 6) / 3, f = (q - 6) % 3;
  if (f == 0) return min(255u, k - 1u - 255u * run);
  return f == 1 ? 0u : 1u;
}

struct RepairWireArgs {
  uint32_t G, k, r, stride, pkt_stride;
  const uint8_t* rep;
  const uint16_t* rep_size;
  const uint16_t* rep_len;
  const uint32_t* sid_base;
  const uint32_t* rid_base;
  uint8_t* out;
  uint32_t* pkt_len;
};

// One workgroup per repair (g, j).  Packet: [0] 1, [1,5) id, [5,7) size, [7, o1) symbol,
// [o1, o2) ids, [o2, o2+2) encoded size, [o2+2, o3) size, [o3, o3+size) symbol (write_repair).
__global__ __launch_bounds__(kWireThreads) void wire_write_repairs(RepairWireArgs a)
{
  const uint32_t p = blockIdx.x;
  const uint32_t g = p / a.r, j = p % a.r;
  const uint32_t symsz = a.rep_len[g];
  const uint32_t sidb = a.sid_base ? a.sid_base[g] : g * a.k;
  const uint32_t rid = (a.rid_base ? a.rid_base[g] : g * a.r) + j;
  const uint32_t esz = a.rep_size[p];
  const uint32_t o1 = 7u + symsz, o2 = o1 + ids_bytes(a.k), o3 = o2 + 4u, total = o3 + symsz;
  const uint8_t* sym = a.rep + static_cast<size_t>(p) * a.stride;
  uint8_t* dst = a.out + static_cast<size_t>(p) * a.pkt_stride;
  // non-symbol bytes (header, id list, trailer); symbol bytes come from s1 / s2 below
  auto meta_byte = [&](uint32_t q) -> uint32_t {
    if (q == 0) return 1u;
    if (q < 5) return (rid >> (8 * (4 - q))) & 0xFFu;
    if (q < 7) return (symsz >> (8 * (6 - q))) & 0xFFu;
    if (q < o2) return ids_byte(a.k, sidb, q - o1);
    if (q < o2 + 2) return (esz >> (8 * (o2 + 1 - q))) & 0xFFu;
    return (symsz >> (8 * (o3 - 1 - q))) & 0xFFu;
  };
  const uint32_t nchunks = (total + 15u) / 16u;
  const uint32_t sh2 = (16u - (o3 & 15u)) & 15u;     // symbol offset of chunk starts in copy 2
  for (uint32_t c = threadIdx.x; c < nchunks; c += kWireThreads) {
    const uint32_t q0 = 16u * c;
    uint4 v;
    if (q0 >= 7u && q0 + 16u <= o1) {                // inside symbol copy 1: offset q0 - 7
      const uint32_t off = q0 - 7u;
      v = load16_shifted(sym + (off & ~15u), 9u, a.stride - (off & ~15u));
    } else if (q0 >= o3 && q0 + 16u <= total) {      // inside symbol copy 2
      const uint32_t off = q0 - o3;
      v = load16_shifted(sym + (off & ~15u), sh2, a.stride - (off & ~15u));
    } else {                                         // boundary chunk: select byte by byte
      const uint4 s1 = slot16(sym, static_cast<int32_t>(q0) - 7, a.stride);
      const uint4 s2 = slot16(sym, static_cast<int32_t>(q0) - static_cast<int32_t>(o3), a.stride);
      v = make_uint4(0, 0, 0, 0);
      for (uint32_t i = 0; i < 16; ++i) {
        const uint32_t q = q0 + i;
        const uint32_t x = q >= total ? 0u
                         : q >= o3 ? get_byte(s2, i)
                         : (q >= 7 && q < o1) ? get_byte(s1, i) : meta_byte(q);
        put_byte(v, i, x);
      }
    }
    *reinterpret_cast<uint4*>(dst + q0) = v;
  }
  if (threadIdx.x == 0) a.pkt_len[p] = total;
}

struct SourceWireArgs {
  uint32_t G, k, stride, pkt_stride;
  const uint8_t* src;
  const uint16_t* src_len;
  const uint32_t* sid_base;
  uint8_t* out;
  uint32_t* pkt_len;
};

// One workgroup per source slot (g, i): [0] 2, [1,5) id, [5,7) size, [7, 7+size) payload.
__global__ __launch_bounds__(kWireThreads) void wire_write_sources(SourceWireArgs a)
{
  const uint32_t p = blockIdx.x;
  const uint32_t g = p / a.k, i = p % a.k;
  const uint32_t len = a.src_len[p];
  const uint32_t sid = (a.sid_base ? a.sid_base[g] : g * a.k) + i;
  const uint32_t total = 7u + len;
  const uint8_t* sym = a.src + static_cast<size_t>(p) * a.stride;
  uint8_t* dst = a.out + static_cast<size_t>(p) * a.pkt_stride;
  const uint32_t nchunks = (total + 15u) / 16u;
  for (uint32_t c = threadIdx.x; c < nchunks; c += kWireThreads) {
    const uint32_t q0 = 16u * c;
    uint4 v;
    if (q0 >= 7u && q0 + 16u <= total) {
      const uint32_t off = q0 - 7u;
      v = load16_shifted(sym + (off & ~15u), 9u, a.stride - (off & ~15u));
    } else {
      v = make_uint4(0, 0, 0, 0);
      for (uint32_t b = 0; b < 16; ++b) {
        const uint32_t q = q0 + b;
        uint32_t x = 0;
        if (q == 0) x = 2u;
        else if (q < 5) x = (sid >> (8 * (4 - q))) & 0xFFu;
        else if (q < 7) x = (len >> (8 * (6 - q))) & 0xFFu;
        else if (q < total) x = sym[q - 7];
        put_byte(v, b, x);
      }
    }
    *reinterpret_cast<uint4*>(dst + q0) = v;
  }
  if (threadIdx.x == 0) a.pkt_len[p] = total;
}

// ---- ingestion --------------------------------------------------------------------------------

struct ReadArgs {
  uint32_t npkts, pkt_stride;
  const uint8_t* pkts;
  const uint32_t* pkt_len;
  uint32_t G, k, r, stride, sid0, rid0;
  uint8_t* src;
  uint16_t* src_len;
  uint8_t* src_mask;
  uint8_t* rep;
  uint16_t* rep_size;
  uint8_t* rep_mask;
  uint8_t* status;
};

// One workgroup per packet.  Every thread parses the header (and a repair's id list) redundantly
// -- uniform control flow, a few dozen bytes -- then the threads copy the symbol into its slot.
__global__ __launch_bounds__(kWireThreads) void wire_read_packets(ReadArgs a)
{
  const uint32_t p = blockIdx.x;
  const uint8_t* pk = a.pkts + static_cast<size_t>(p) * a.pkt_stride;
  const uint32_t len = min(a.pkt_len[p], a.pkt_stride);
  uint32_t pos = 0;
  bool over = false;
  auto rd = [&](uint32_t n) -> uint32_t {      // big-endian read of n bytes (packetizer read<T>)
    if (len - pos < n || pos > len) { over = true; return 0u; }
    uint32_t x = 0;
    for (uint32_t b = 0; b < n; ++b) x = (x << 8) | pk[pos + b];
    pos += n;
    return x;
  };
  uint32_t st;
  if (len == 0) {
    st = NTC_PKT_OVERFLOW;
  } else {
    const uint32_t ty = pk[0];
    pos = 1;
    if (ty == 0) st = NTC_PKT_ACK;
    else if (ty != 1 && ty != 2) st = NTC_PKT_BAD_TYPE;
    else {
      const uint32_t id = rd(4);
      const uint32_t symsz = rd(2);
      if (over || len - pos < symsz) {
        st = NTC_PKT_OVERFLOW;
      } else {
        pos += symsz;
        uint32_t d, esz = 0;
        bool full = true;
        if (ty == 2) {
          d = id - a.sid0;
          st = static_cast<uint64_t>(d) >= static_cast<uint64_t>(a.G) * a.k ? NTC_PKT_OUT_OF_BATCH
             : symsz > a.stride ? NTC_PKT_TOO_LARGE : NTC_PKT_SOURCE;
        } else {
          // read_ids (packetizer.hh:312-352): the set {first + running sums of the deltas}
          const uint32_t count = rd(2);
          uint32_t first = 0, ones = 0;
          bool step_ok = true;
          if (count != 0) {
            first = rd(4);
            for (uint32_t e = 0; e + 1 < count && !over; ++e) {
              const uint32_t run = rd(1), v = rd(2);
              if (run == 0) continue;
              if (v == 1) ones += run;
              else if (v != 0) step_ok = false;
            }
          }
          esz = rd(2);
          d = id - a.rid0;
          const uint32_t g = d / a.r;
          // (ids do not wrap inside a generation: gpu.h layout contract)
          full = count != 0 && step_ok && first == a.sid0 + g * a.k && ones + 1 == a.k &&
                 first <= 0xFFFFFFFFu - (a.k - 1u);
          st = over ? NTC_PKT_OVERFLOW
             : static_cast<uint64_t>(d) >= static_cast<uint64_t>(a.G) * a.r ? NTC_PKT_OUT_OF_BATCH
             : symsz > a.stride ? NTC_PKT_TOO_LARGE
             : !full ? NTC_PKT_NOT_GENERATION : NTC_PKT_REPAIR;
        }
        if (st == NTC_PKT_SOURCE || st == NTC_PKT_REPAIR) {
          uint8_t* dst = (st == NTC_PKT_SOURCE ? a.src : a.rep) + static_cast<size_t>(d) * a.stride;
          // payload at packet offset 7: chunk c of the slot = packet bytes [7 + 16c, +16)
          for (uint32_t c = threadIdx.x; c < a.stride / 16u; c += kWireThreads) {
            const uint32_t q0 = 16u * c;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (q0 < symsz) {
              v = load16_shifted(pk + q0, 7u, a.pkt_stride - q0);
              if (q0 + 16u > symsz)
                for (uint32_t b = symsz - q0; b < 16; ++b) put_byte(v, b, 0u);
            }
            *reinterpret_cast<uint4*>(dst + q0) = v;
          }
          if (threadIdx.x == 0) {
            if (st == NTC_PKT_SOURCE) {
              a.src_len[d] = static_cast<uint16_t>(symsz);
              a.src_mask[d] = 1;
            } else {
              a.rep_size[d] = static_cast<uint16_t>(esz);
              a.rep_mask[d] = 1;
            }
          }
        }
      }
    }
  }
  if (threadIdx.x == 0) a.status[p] = static_cast<uint8_t>(st);
}

// ---- packed <-> slot layout (host-resident batches) -------------------------------------------

struct PackArgs {
  uint32_t G, k, stride, want, row0;
  int zero_rest;                 // unpack: zero the slots not selected
  const uint8_t* mask;
  const uint32_t* row_base;
  const uint8_t* from;
  uint8_t* to;
};

// One workgroup per slot (g, i).  The slot is selected when (mask != 0) == want; its packed row
// is row_base[g] - row0 + (selected slots of g before i), counted with one block-wide
// __syncthreads_count per 256 slots.  UNPACK copies packed row -> slot, PACK slot -> packed row.
template <bool UNPACK>
__global__ __launch_bounds__(kWireThreads) void slot_pack(PackArgs a)
{
  const uint32_t p = blockIdx.x;
  const uint32_t g = p / a.k, i = p % a.k;
  const uint8_t* m = a.mask + static_cast<size_t>(g) * a.k;
  const bool sel = (m[i] != 0) == (a.want != 0);          // uniform over the block
  const uint32_t n16 = a.stride / 16u;
  if (!sel) {
    if (UNPACK && a.zero_rest) {
      uint8_t* dst = a.to + static_cast<size_t>(p) * a.stride;
      for (uint32_t c = threadIdx.x; c < n16; c += kWireThreads)
        *reinterpret_cast<uint4*>(dst + 16u * c) = make_uint4(0, 0, 0, 0);
    }
    return;
  }
  uint32_t rank = 0;
  for (uint32_t j0 = 0; j0 < i; j0 += kWireThreads) {
    const uint32_t j = j0 + threadIdx.x;
    rank += __syncthreads_count(j < i && (m[j] != 0) == (a.want != 0));
  }
  const size_t row = static_cast<size_t>(a.row_base[g] - a.row0 + rank);
  const uint8_t* src = UNPACK ? a.from + row * a.stride : a.from + static_cast<size_t>(p) * a.stride;
  uint8_t* dst = UNPACK ? a.to + static_cast<size_t>(p) * a.stride : a.to + row * a.stride;
  for (uint32_t c = threadIdx.x; c < n16; c += kWireThreads)
    *reinterpret_cast<uint4*>(dst + 16u * c) = *reinterpret_cast<const uint4*>(src + 16u * c);
}

uint32_t host_ids_bytes(uint32_t k) { return k == 0 ? 2u : 6u + 3u * ((k - 1u + 254u) / 255u); }

int pack_launch(bool unpack, ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t stride,
                const uint8_t* mask, uint32_t want, const uint32_t* row_base, uint32_t row0,
                const uint8_t* from, uint8_t* to, int zero_rest, void* stream)
{
  if (!e || !mask || !row_base || !from || !to) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0) return fail(NTC_GPU_EINVAL, "G and k must be > 0");
  if (stride == 0 || stride % 16 != 0 || stride > 65536)
    return fail(NTC_GPU_EINVAL, "stride must be a non-zero multiple of 16, <= 65536");
  const uint64_t n = static_cast<uint64_t>(G) * k;
  if (n > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "too many slots for one launch");
  (void)hipSetDevice(e->device);
  PackArgs a{G, k, stride, want, row0, zero_rest, mask, row_base, from, to};
  if (unpack)
    hipLaunchKernelGGL(slot_pack<true>, dim3(static_cast<uint32_t>(n)), dim3(kWireThreads), 0,
                       static_cast<hipStream_t>(stream), a);
  else
    hipLaunchKernelGGL(slot_pack<false>, dim3(static_cast<uint32_t>(n)), dim3(kWireThreads), 0,
                       static_cast<hipStream_t>(stream), a);
  return hip_check(hipGetLastError(), unpack ? "slot_unpack launch" : "slot_pack launch");
}

}  // namespace
}  // namespace ntcgpu

using namespace ntcgpu;

extern "C" {

uint32_t ntc_gf256_repair_packet_bytes(uint32_t k, uint32_t stride)
{
  const uint32_t n = 11u + 2u * stride + host_ids_bytes(k);
  return (n + 15u) & ~15u;
}

int ntc_gf256_write_repairs(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r, uint32_t stride,
                            const uint8_t* rep, const uint16_t* rep_size, const uint16_t* rep_len,
                            const uint32_t* sid_base, const uint32_t* rid_base, uint8_t* out,
                            uint32_t pkt_stride, uint32_t* pkt_len, void* stream)
{
  if (!e || !rep || !rep_size || !rep_len || !out || !pkt_len) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0 || r == 0) return fail(NTC_GPU_EINVAL, "G, k and r must be > 0");
  if (stride % 16 != 0 || stride > 65536) return fail(NTC_GPU_EINVAL, "stride must be a multiple of 16, <= 65536");
  if (pkt_stride % 16 != 0 || pkt_stride < ntc_gf256_repair_packet_bytes(k, stride))
    return fail(NTC_GPU_EINVAL, "pkt_stride must be a multiple of 16 >= ntc_gf256_repair_packet_bytes(k, stride)");
  const uint64_t n = static_cast<uint64_t>(G) * r;
  if (n > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "too many packets for one launch");
  (void)hipSetDevice(e->device);
  RepairWireArgs a{G, k, r, stride, pkt_stride, rep, rep_size, rep_len, sid_base, rid_base, out, pkt_len};
  hipLaunchKernelGGL(wire_write_repairs, dim3(static_cast<uint32_t>(n)), dim3(kWireThreads), 0,
                     static_cast<hipStream_t>(stream), a);
  return hip_check(hipGetLastError(), "wire_write_repairs launch");
}

int ntc_gf256_write_sources(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t stride,
                            const uint8_t* src, const uint16_t* src_len, const uint32_t* sid_base,
                            uint8_t* out, uint32_t pkt_stride, uint32_t* pkt_len, void* stream)
{
  if (!e || !src || !src_len || !out || !pkt_len) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0) return fail(NTC_GPU_EINVAL, "G and k must be > 0");
  if (stride % 16 != 0 || stride > 65536) return fail(NTC_GPU_EINVAL, "stride must be a multiple of 16, <= 65536");
  if (pkt_stride % 16 != 0 || pkt_stride < ((7u + stride + 15u) & ~15u))
    return fail(NTC_GPU_EINVAL, "pkt_stride must be a multiple of 16 >= 7 + stride");
  const uint64_t n = static_cast<uint64_t>(G) * k;
  if (n > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "too many packets for one launch");
  (void)hipSetDevice(e->device);
  SourceWireArgs a{G, k, stride, pkt_stride, src, src_len, sid_base, out, pkt_len};
  hipLaunchKernelGGL(wire_write_sources, dim3(static_cast<uint32_t>(n)), dim3(kWireThreads), 0,
                     static_cast<hipStream_t>(stream), a);
  return hip_check(hipGetLastError(), "wire_write_sources launch");
}

static int read_packets_impl(bool reset, ntc_gf256_engine* e, uint32_t npkts, const uint8_t* pkts,
                             uint32_t pkt_stride, const uint32_t* pkt_len, uint32_t G, uint32_t k,
                             uint32_t r, uint32_t stride, uint32_t sid0, uint32_t rid0, uint8_t* src,
                             uint16_t* src_len, uint8_t* src_mask, uint8_t* rep, uint16_t* rep_size,
                             uint8_t* rep_mask, uint8_t* status, void* stream)
{
  if (!e || !src || !src_len || !src_mask || !rep || !rep_size || !rep_mask)
    return fail(NTC_GPU_EINVAL, "NULL argument");
  if (npkts && (!pkts || !pkt_len || !status)) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0 || r == 0) return fail(NTC_GPU_EINVAL, "G, k and r must be > 0");
  if (stride % 16 != 0 || stride > 65536) return fail(NTC_GPU_EINVAL, "stride must be a multiple of 16, <= 65536");
  if (pkt_stride % 16 != 0 || pkt_stride == 0) return fail(NTC_GPU_EINVAL, "pkt_stride must be a non-zero multiple of 16");
  if (npkts > 0x7FFFFFFFu) return fail(NTC_GPU_EUNSUPPORTED, "too many packets for one launch");
  (void)hipSetDevice(e->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t nk = static_cast<size_t>(G) * k, nr = static_cast<size_t>(G) * r;
  int rc;
  if (reset) {
    if ((rc = hip_check(hipMemsetAsync(src_mask, 0, nk, st), "reset src_mask"))) return rc;
    if ((rc = hip_check(hipMemsetAsync(src_len, 0, 2 * nk, st), "reset src_len"))) return rc;
    if ((rc = hip_check(hipMemsetAsync(rep_mask, 0, nr, st), "reset rep_mask"))) return rc;
    if ((rc = hip_check(hipMemsetAsync(rep_size, 0, 2 * nr, st), "reset rep_size"))) return rc;
  }
  if (npkts == 0) return NTC_GPU_OK;
  ReadArgs a{npkts, pkt_stride, pkts, pkt_len, G, k, r, stride, sid0, rid0,
             src, src_len, src_mask, rep, rep_size, rep_mask, status};
  hipLaunchKernelGGL(wire_read_packets, dim3(npkts), dim3(kWireThreads), 0, st, a);
  return hip_check(hipGetLastError(), "wire_read_packets launch");
}

int ntc_gf256_read_packets(ntc_gf256_engine* e, uint32_t npkts, const uint8_t* pkts,
                           uint32_t pkt_stride, const uint32_t* pkt_len, uint32_t G, uint32_t k,
                           uint32_t r, uint32_t stride, uint32_t sid0, uint32_t rid0, uint8_t* src,
                           uint16_t* src_len, uint8_t* src_mask, uint8_t* rep, uint16_t* rep_size,
                           uint8_t* rep_mask, uint8_t* status, void* stream)
{
  return read_packets_impl(true, e, npkts, pkts, pkt_stride, pkt_len, G, k, r, stride, sid0, rid0, src,
                           src_len, src_mask, rep, rep_size, rep_mask, status, stream);
}

int ntc_gf256_read_packets_append(ntc_gf256_engine* e, uint32_t npkts, const uint8_t* pkts,
                                  uint32_t pkt_stride, const uint32_t* pkt_len, uint32_t G, uint32_t k,
                                  uint32_t r, uint32_t stride, uint32_t sid0, uint32_t rid0, uint8_t* src,
                                  uint16_t* src_len, uint8_t* src_mask, uint8_t* rep, uint16_t* rep_size,
                                  uint8_t* rep_mask, uint8_t* status, void* stream)
{
  return read_packets_impl(false, e, npkts, pkts, pkt_stride, pkt_len, G, k, r, stride, sid0, rid0, src,
                           src_len, src_mask, rep, rep_size, rep_mask, status, stream);
}

int ntc_gf256_unpack_slots(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t stride,
                           const uint8_t* packed, const uint32_t* row_base, uint32_t row0,
                           const uint8_t* mask, uint8_t want, uint8_t* slots, int zero_rest,
                           void* stream)
{
  return pack_launch(true, e, G, k, stride, mask, want, row_base, row0, packed, slots, zero_rest,
                     stream);
}

int ntc_gf256_pack_slots(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t stride,
                         const uint8_t* slots, const uint8_t* mask, uint8_t want,
                         const uint32_t* row_base, uint32_t row0, uint8_t* packed, void* stream)
{
  return pack_launch(false, e, G, k, stride, mask, want, row_base, row0, slots, packed, 0, stream);
}

}  // extern "C"
