// ntc_gfw.hip -- GF(2^w) for every field size netcode supports, w in {4, 8, 16, 32}
// (galois_field.hh:35-44 gf_init_easy(&gf, w)).
//
// The fields are gf-complete's defaults: primitive polynomials 0x13 (w=4), 0x11D (w=8), 0x1100B
// (w=16), x^32 + 0x400007 (w=32).  Region semantics of multiply_region.w32: w=4 multiplies every
// nibble, w=8 every byte, w=16 / w=32 every little-endian 16- / 32-bit word of the region.
//
// Device work is shift-and-add on packed elements: a dword holds 8 / 4 / 2 / 1 elements and xtime
// (multiply by alpha) is a shift plus a reduction constant for all of them at once (packed 16-bit
// shifts for w = 16, an arithmetic-shift mask for w = 32).  The batched combine walks the powers
// x * alpha^t once per input dword and adds each into the rows whose coefficient has bit t set --
// a wave-uniform 0 / -1 mask per (row, t), so one AND-XOR per (row, t, dword) -- which amortises
// the w xtime steps over up to 8 rows.  This serves the per-packet C ABI (libntc.so) for w != 8
// and the batched combine for any w; the GF(2^8) batch path keeps its dedicated kernels
// (ntc_gf256.hip).  Host-side scalar arithmetic (coefficient, multiply, invert, multiply_size) is
// the carry-less product reduced by the same polynomials.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "engine.hh"
#include "netcode/gpu.h"

namespace ntcgpu {
namespace {

// byte-packed fields (w = 4, 8): per-element shift mask, the elements' top bits, shift to bit 0
template <int W> struct Packed;
template <> struct Packed<4> {
  static constexpr uint32_t keep = 0xEEEEEEEEu, top = 0x11111111u, shift = 3;
};
template <> struct Packed<8> {
  static constexpr uint32_t keep = 0xFEFEFEFEu, top = 0x01010101u, shift = 7;
};

// alpha * x for every element packed in x
template <int W>
__device__ __forceinline__ uint32_t xtime(uint32_t y)
{
  if constexpr (W == 32) {
    return (y << 1) ^ (static_cast<uint32_t>(static_cast<int32_t>(y) >> 31) & 0x00400007u);
  } else if constexpr (W == 16) {
    // two u16 lanes: per-half shift (no carry across) and per-half sign mask
    typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
    typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 h = __builtin_bit_cast(u16x2, y);
    const u16x2 sh = h << static_cast<uint16_t>(1);
    const i16x2 sg = __builtin_bit_cast(i16x2, y) >> static_cast<int16_t>(15);
    return __builtin_bit_cast(uint32_t, sh) ^ (__builtin_bit_cast(uint32_t, sg) & 0x100B100Bu);
  } else {
    const uint32_t t = (y >> Packed<W>::shift) & Packed<W>::top;
    uint32_t red;
    if constexpr (W == 4) {
      red = t | (t << 1);                                                      // * 0x3
    } else {                                                                   // * 0x1D, per u16 half
      typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
      const u16x2 k = {0x1D, 0x1D};
      red = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, t) * k);
    }
    return ((y << 1) & Packed<W>::keep) ^ red;
  }
}

// c * x for every element packed in x (the loop ends after c's top bit; uniform when c is).
template <int W>
__device__ __forceinline__ uint32_t mulw(uint32_t c, uint32_t x)
{
  uint32_t r = 0, y = x;
  for (int t = 0; t < W; ++t) {
    const uint32_t ct = c >> t;
    if (ct == 0) break;
    if (ct & 1u) r ^= y;
    y = xtime<W>(y);
  }
  return r;
}

struct CombineArgs {
  uint32_t G, k, rows, stride;
  const uint8_t* in;       // [G][k][stride]
  const uint32_t* coef;    // [G][k][rows]
  uint8_t* out;            // [G][rows][stride]
};

// One wave per (generation, 1 KiB column span, group of RB rows); a lane owns 16 bytes of the span
// for all RB rows.  Per input: the 4 dwords walk x, x*alpha, ..., x*alpha^(W-1) and every row adds
// the powers its coefficient selects (mask 0 / -1 from bit t of the wave-uniform coefficient).
// The next input's 16 bytes are loaded before this one's powers are walked.
constexpr uint32_t kGfwSpan = 1024;

template <int W, int RB>
__global__ __launch_bounds__(256) void gfw_combine(CombineArgs a, uint32_t nspan, uint32_t ngrp)
{
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t per_g = nspan * ngrp;
  if (wave >= a.G * per_g) return;
  const uint32_t g = wave / per_g, rem = wave % per_g;
  const uint32_t span = rem % nspan, r0 = (rem / nspan) * RB;
  const uint32_t col = span * kGfwSpan + 16u * lane;
  const bool act = col < a.stride;
  const uint32_t nr = a.rows - r0 < static_cast<uint32_t>(RB) ? a.rows - r0 : static_cast<uint32_t>(RB);
  const uint8_t* in = a.in + static_cast<size_t>(g) * a.k * a.stride + (act ? col : 0u);
  const uint32_t* cf = a.coef + static_cast<size_t>(g) * a.k * a.rows + r0;
  uint32_t acc[RB][4];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[r][d] = 0;
  uint4 nx = act ? *reinterpret_cast<const uint4*>(in) : make_uint4(0, 0, 0, 0);
  for (uint32_t i = 0; i < a.k; ++i) {
    uint32_t y[4] = {nx.x, nx.y, nx.z, nx.w};
    if (act && i + 1 < a.k) nx = *reinterpret_cast<const uint4*>(in + static_cast<size_t>(i + 1) * a.stride);
    uint32_t c[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
      c[r] = static_cast<uint32_t>(r) < nr ? __builtin_amdgcn_readfirstlane(cf[static_cast<size_t>(i) * a.rows + r]) : 0u;
    if constexpr (W < 32) {
#pragma unroll
      for (int r = 0; r < RB; ++r) c[r] &= (1u << W) - 1u;
    }
    uint32_t any = 0;
#pragma unroll
    for (int r = 0; r < RB; ++r) any |= c[r];
    if (any == 0) continue;                             // wave-uniform
#pragma unroll
    for (int t = 0; t < W; ++t) {
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const uint32_t m = 0u - ((c[r] >> t) & 1u);
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[r][d] = __builtin_amdgcn_bitop3_b32(acc[r][d], y[d], m, 0x78);   // a ^ (y & m)
      }
      if (t + 1 < W) {
#pragma unroll
        for (int d = 0; d < 4; ++d) y[d] = xtime<W>(y[d]);
      }
    }
  }
  if (!act) return;
#pragma unroll
  for (int r = 0; r < RB; ++r)
    if (static_cast<uint32_t>(r) < nr)
      *reinterpret_cast<uint4*>(a.out + (static_cast<size_t>(g) * a.rows + r0 + r) * a.stride + col) =
          make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}

// Four-Russians form (round 6, the default for groups of 8 rows): per input dword the 16 XOR
// combinations of each group of four powers x*alpha^(4g) .. x*alpha^(4g+3) are built once (w - 1
// xtime steps + 11 XORs per group), and a row adds one table entry per group -- the entry chosen by the nibble of its
// wave-uniform coefficient through VGPR-relative addressing (gfw_fr_lookup, generated by
// tools/gen_gfw_fr.py).  Per (row, input dword): w/4 indexed XORs instead of the masked form's w
// AND-XORs.  A lane owns D dwords (the table takes 16 * (w/4) * D VGPRs, <= 128).
template <int W> struct FrGeom {
  static constexpr int G = W / 4 > 0 ? W / 4 : 1;
  static constexpr int D = W == 4 ? 4 : W == 32 ? 1 : 2;
  static constexpr int NT = 16 * G * D;
  static constexpr uint32_t SPAN = 256u * D;
};

#include "gfw_fr_lookup.inc"

// a wave-uniform load through the scalar unit (constant address space)
template <typename T>
__device__ __forceinline__ T const_load(const void* p)
{
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

// alpha * x with every shift amount and mask in a VGPR (opaque to the compiler, so it cannot
// fold them back into inline constants or SGPR operands, whose VALU forms issue at half rate on
// gfx950 -- DESIGN §3 "Issue rates by instruction form")
template <int W> struct XtimeV {
  uint32_t a, b, k;        // w = 16: (1,1), (15,15), 0x100B100B; w = 32: 1, 31, 0x00400007
  __device__ __forceinline__ XtimeV()
  {
    constexpr uint32_t A = W == 16 ? 0x00010001u : 1u, B = W == 16 ? 0x000F000Fu : 31u;
    constexpr uint32_t K = W == 16 ? 0x100B100Bu : 0x00400007u;
    asm volatile("v_mov_b32 %0, %3\n" "v_mov_b32 %1, %4\n" "v_mov_b32 %2, %5\n"
                 : "=v"(a), "=v"(b), "=v"(k) : "i"(A), "i"(B), "i"(K));
  }
  __device__ __forceinline__ uint32_t operator()(uint32_t y) const
  {
    if constexpr (W == 16) {
      typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
      typedef int16_t i16x2 __attribute__((ext_vector_type(2)));
      const u16x2 sh = __builtin_bit_cast(u16x2, y) << __builtin_bit_cast(u16x2, a);
      const i16x2 sg = __builtin_bit_cast(i16x2, y) >> __builtin_bit_cast(i16x2, b);
      return __builtin_amdgcn_bitop3_b32(__builtin_bit_cast(uint32_t, sh), __builtin_bit_cast(uint32_t, sg), k, 0x78);
    } else {
      const uint32_t sg = static_cast<uint32_t>(static_cast<int32_t>(y) >> b);
      return __builtin_amdgcn_bitop3_b32(y << a, sg, k, 0x78);
    }
  }
};
template <int W> struct XtimeC {      // w = 4, 8: the packed-byte forms as they are
  __device__ __forceinline__ uint32_t operator()(uint32_t y) const { return xtime<W>(y); }
};

template <int D> struct LaneVec;
template <> struct LaneVec<1> {
  typedef uint32_t T;
  static __device__ __forceinline__ void get(const T& v, uint32_t (&x)[1]) { x[0] = v; }
  static __device__ __forceinline__ T make(const uint32_t (&x)[1]) { return x[0]; }
};
template <> struct LaneVec<2> {
  typedef uint2 T;
  static __device__ __forceinline__ void get(const T& v, uint32_t (&x)[2]) { x[0] = v.x; x[1] = v.y; }
  static __device__ __forceinline__ T make(const uint32_t (&x)[2]) { return make_uint2(x[0], x[1]); }
};
template <> struct LaneVec<4> {
  typedef uint4 T;
  static __device__ __forceinline__ void get(const T& v, uint32_t (&x)[4])
  {
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
  static __device__ __forceinline__ T make(const uint32_t (&x)[4]) { return make_uint4(x[0], x[1], x[2], x[3]); }
};

// One wave per (generation, SPAN-byte column span, group of RB rows); a lane owns 4*D bytes.
template <int W, int RB>
__global__ __launch_bounds__(256) void gfw_combine_fr(CombineArgs a, uint32_t nspan, uint32_t ngrp)
{
  constexpr int G = FrGeom<W>::G, D = FrGeom<W>::D, NT = FrGeom<W>::NT;
  typedef typename LaneVec<D>::T V;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t per_g = nspan * ngrp;
  if (wave >= a.G * per_g) return;
  const uint32_t g = wave / per_g, rem = wave % per_g;
  const uint32_t span = rem % nspan, r0 = (rem / nspan) * RB;
  const uint32_t col = span * FrGeom<W>::SPAN + 4u * D * lane;
  const bool act = col < a.stride;                    // stride % 16 == 0: all D dwords or none
  const uint32_t nr = a.rows - r0 < static_cast<uint32_t>(RB) ? a.rows - r0 : static_cast<uint32_t>(RB);
  const uint8_t* in = a.in + static_cast<size_t>(g) * a.k * a.stride + (act ? col : 0u);
  const uint32_t* cf = a.coef + static_cast<size_t>(g) * a.k * a.rows + r0;
  uint32_t acc[RB][D];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int d = 0; d < D; ++d) acc[r][d] = 0;
  // coefficients through the scalar unit, one input ahead (rows past the group's last read its
  // last row's word and are zeroed)
  typedef uint32_t CV __attribute__((ext_vector_type(RB)));
  auto coefs = [&](uint32_t i, uint32_t (&c)[RB]) {
    const uint32_t* p = cf + static_cast<size_t>(i) * a.rows;
    if (nr == static_cast<uint32_t>(RB)) {             // the group's RB words in one scalar load
      const CV v = const_load<CV>(p);
#pragma unroll
      for (int r = 0; r < RB; ++r) c[r] = v[r];
    } else {
#pragma unroll
      for (int r = 0; r < RB; ++r)
        c[r] = static_cast<uint32_t>(r) < nr ? const_load<uint32_t>(p + r) : 0u;
    }
  };
  uint32_t cn[RB];
  coefs(0, cn);
  // (16 rows: the constant forms, whose operands need no VGPRs -- measured as fast at 8 rows)
  const typename std::conditional<(W >= 16 && RB < 16), XtimeV<W>, XtimeC<W>>::type xtv;
  // inputs PF ahead in registers (a wave's work per input is short next to the memory latency)
  constexpr int PF = RB == 16 && D == 2 ? 1 : D == 4 ? 2 : 3;   // (w = 16 x 16 rows: 3 waves per SIMD need <= 168 VGPRs)
  V nx[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j)
    nx[j] = act && static_cast<uint32_t>(j) < a.k ? *reinterpret_cast<const V*>(in + static_cast<size_t>(j) * a.stride) : V{};
  for (uint32_t i = 0; i < a.k; ++i) {
    uint32_t x[D];
    LaneVec<D>::get(nx[0], x);
#pragma unroll
    for (int j = 0; j + 1 < PF; ++j) nx[j] = nx[j + 1];
    if (act && i + PF < a.k) nx[PF - 1] = *reinterpret_cast<const V*>(in + static_cast<size_t>(i + PF) * a.stride);
    uint32_t c[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) c[r] = cn[r];
    if (i + 1 < a.k) coefs(i + 1, cn);
    if constexpr (W < 32) {
#pragma unroll
      for (int r = 0; r < RB; ++r) c[r] &= (1u << W) - 1u;
    }
    uint32_t any = 0;
#pragma unroll
    for (int r = 0; r < RB; ++r) any |= c[r];
    if (any == 0) continue;                             // wave-uniform
    uint32_t T[NT];
    // the D dwords' power chains side by side (independent: each step of one hides the other's latency)
    uint32_t y[D];
#pragma unroll
    for (int d = 0; d < D; ++d) y[d] = x[d];
#pragma unroll
    for (int q = 0; q < G; ++q) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          uint32_t* t = T + (d * G + q) * 16;
          if (j == 0) t[0] = 0;
          t[1 << j] = y[d];
          if (j < 3 || q + 1 < G) y[d] = xtv(y[d]);
        }
      }
#pragma unroll
      for (int d = 0; d < D; ++d) {
        uint32_t* t = T + (d * G + q) * 16;
#ifdef NTC_GFW_ABL_NOTABLE
#pragma unroll
        for (int m = 0; m < 16; ++m) t[m] = x[d] + m;
        continue;
#endif
        t[3] = t[1] ^ t[2];
        t[5] = t[4] ^ t[1];
        t[6] = t[4] ^ t[2];
        t[7] = t[4] ^ t[3];
#pragma unroll
        for (int m = 1; m < 8; ++m) t[8 + m] = t[8] ^ t[m];
      }
    }
#if defined(NTC_GFW_ABL_NOLOOKUP)    // timing-only ablations (tools/build_variant.sh -D...)
#pragma unroll
    for (int j = 0; j < NT; ++j) asm volatile("" :: "v"(T[j]));
#pragma unroll
    for (int r = 0; r < RB; ++r) acc[r][0] ^= c[r];
#else
    gfw_fr_lookup<W, RB>(acc, T, c);
#endif
  }
  if (!act) return;
#pragma unroll
  for (int r = 0; r < RB; ++r)
    if (static_cast<uint32_t>(r) < nr)
      *reinterpret_cast<V*>(a.out + (static_cast<size_t>(g) * a.rows + r0 + r) * a.stride + col) =
          LaneVec<D>::make(acc[r]);
}

// dst[0..len) = c * src (+ dst); word boundaries relative to the region start; a partial last word
// reads missing bytes as zero and writes only bytes inside len.
template <int W>
__global__ __launch_bounds__(256) void gfw_region(const uint8_t* __restrict__ src, uint8_t* dst,
                                                  uint64_t len, uint32_t c, int add)
{
  const uint64_t d = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  const uint64_t b0 = 4 * d;
  if (b0 >= len) return;
  const uint32_t nb = static_cast<uint32_t>(len - b0 < 4 ? len - b0 : 4);
  uint32_t x = 0;
  for (uint32_t b = 0; b < nb; ++b) x |= static_cast<uint32_t>(src[b0 + b]) << (8 * b);
  const uint32_t y = mulw<W>(c, x);
  for (uint32_t b = 0; b < nb; ++b) {
    const uint8_t o = static_cast<uint8_t>(y >> (8 * b));
    dst[b0 + b] = add ? static_cast<uint8_t>(dst[b0 + b] ^ o) : o;
  }
}

bool valid_w(uint32_t w) { return w == 4 || w == 8 || w == 16 || w == 32; }

uint64_t host_poly(uint32_t w)
{
  return w == 4 ? 0x13u : w == 8 ? 0x11Du : w == 16 ? 0x1100Bu : 0x100400007ull;
}

}  // namespace
}  // namespace ntcgpu

using namespace ntcgpu;

extern "C" {

uint32_t ntc_gf_multiply(uint32_t w, uint32_t a, uint32_t b)
{
  if (!valid_w(w) || a == 0 || b == 0) return 0;
  uint64_t r = 0;
  for (uint32_t i = 0; i < w; ++i)
    if ((b >> i) & 1u) r ^= static_cast<uint64_t>(a) << i;
  const uint64_t p = host_poly(w);
  for (int i = 2 * static_cast<int>(w) - 2; i >= static_cast<int>(w); --i)
    if ((r >> i) & 1u) r ^= p << (i - static_cast<int>(w));
  return static_cast<uint32_t>(r);
}

uint32_t ntc_gf_invert(uint32_t w, uint32_t a)
{
  if (!valid_w(w) || a == 0) return 0;
  uint32_t res = 1, base = a;
  uint64_t e = (w == 32 ? 0xFFFFFFFFull : ((1ull << w) - 1)) - 1;   // a^(2^w - 2)
  while (e) {
    if (e & 1) res = ntc_gf_multiply(w, res, base);
    base = ntc_gf_multiply(w, base, base);
    e >>= 1;
  }
  return res;
}

uint32_t ntc_gf_coefficient(uint32_t w, uint32_t repair_id, uint32_t src_id)
{
  if (!valid_w(w)) return 0;
  const uint32_t res = ((repair_id + 1u) + (src_id + 1u)) * (repair_id + 1u);
  if (w == 32) return res == 0 ? 1u : res;
  return res % ((1u << w) - 1u) + 1u;
}

uint16_t ntc_gf_multiply_size(uint32_t w, uint16_t size, uint32_t c)
{
  if (!valid_w(w) || size == 0 || c == 0) return 0;
  if (w == 4) {          // the u16's four nibbles, each multiplied by c
    uint32_t r = 0;
    for (int n = 0; n < 4; ++n) r |= ntc_gf_multiply(4, c, (size >> (4 * n)) & 15u) << (4 * n);
    return static_cast<uint16_t>(r);
  }
  if (w == 8) return static_cast<uint16_t>(ntc_gf_multiply(8, c, size & 0xFFu) |
                                           (ntc_gf_multiply(8, c, size >> 8) << 8));
  return static_cast<uint16_t>(ntc_gf_multiply(w, size, c));   // w = 32: truncated
}

int ntc_gf_combine_batch(ntc_gf256_engine* e, uint32_t w, uint32_t G, uint32_t k, uint32_t rows,
                         uint32_t stride, const uint8_t* in, const uint32_t* coef, uint8_t* out,
                         void* stream)
{
  if (!e || !in || !coef || !out) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (!valid_w(w)) return fail(NTC_GPU_EINVAL, "w must be 4, 8, 16 or 32");
  if (G == 0 || k == 0 || rows == 0) return fail(NTC_GPU_EINVAL, "G, k and rows must be > 0");
  if (stride == 0 || stride % 16 != 0) return fail(NTC_GPU_EINVAL, "stride must be a non-zero multiple of 16");
  // rows per wave: 8, or the next power of two covering fewer rows (16 for the table lookups)
  const uint32_t rbm = rows >= 8 ? 8 : rows > 2 ? 4 : rows;
  // the table lookups pay for their table build only over a full group of 8 rows: with 1, 2 or 4
  // rows per wave the masked form is as fast or faster (profiles/r06/gfw/rows_1_2_4.txt; the per-packet
  // C ABI combines one row per generation).  NTC_GFW_KERNEL=mask / fr forces one form.
  const char* form = std::getenv("NTC_GFW_KERNEL");
  const bool fr = form && std::strcmp(form, "mask") == 0 ? false
                : form && std::strcmp(form, "fr") == 0 ? true : rbm == 8;
  // with 16 rows or more the lookups take 16 rows per wave: the table build is shared by twice
  // the rows (176 VGPRs at w = 16: 2 waves per SIMD)
  const uint32_t rb = fr && rows >= 16 ? 16 : rbm;
  const uint32_t spanb = !fr ? kGfwSpan : w == 4 ? FrGeom<4>::SPAN : w == 8 ? FrGeom<8>::SPAN
                       : w == 16 ? FrGeom<16>::SPAN : FrGeom<32>::SPAN;
  const uint32_t nspan = (stride + spanb - 1) / spanb, ngrp = (rows + rb - 1) / rb;
  const uint64_t waves = static_cast<uint64_t>(G) * nspan * ngrp;
  const uint64_t blocks = (waves + 3) / 4;
  if (blocks > 0x7FFFFFFFull || waves > 0xFFFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "batch too large for one launch");
  (void)hipSetDevice(e->device);
  CombineArgs a{G, k, rows, stride, in, coef, out};
  using Fn = void (*)(CombineArgs, uint32_t, uint32_t);
  Fn fn;
  switch (w * 32 + rb) {
#define NTC_GFW_CASE(W_, RB_) case W_ * 32 + RB_: fn = fr ? gfw_combine_fr<W_, RB_> : gfw_combine<W_, RB_>; break;
#define NTC_GFW_CASE16(W_) case W_ * 32 + 16: fn = gfw_combine_fr<W_, 16>; break;
    NTC_GFW_CASE(4, 1) NTC_GFW_CASE(4, 2) NTC_GFW_CASE(4, 4) NTC_GFW_CASE(4, 8) NTC_GFW_CASE16(4)
    NTC_GFW_CASE(8, 1) NTC_GFW_CASE(8, 2) NTC_GFW_CASE(8, 4) NTC_GFW_CASE(8, 8) NTC_GFW_CASE16(8)
    NTC_GFW_CASE(16, 1) NTC_GFW_CASE(16, 2) NTC_GFW_CASE(16, 4) NTC_GFW_CASE(16, 8) NTC_GFW_CASE16(16)
    NTC_GFW_CASE(32, 1) NTC_GFW_CASE(32, 2) NTC_GFW_CASE(32, 4) NTC_GFW_CASE(32, 8) NTC_GFW_CASE16(32)
#undef NTC_GFW_CASE
#undef NTC_GFW_CASE16
    default: return fail(NTC_GPU_EINVAL, "w must be 4, 8, 16 or 32");
  }
  hipLaunchKernelGGL(fn, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a, nspan, ngrp);
  return hip_check(hipGetLastError(), "gfw_combine launch");
}

int ntc_gf_region_multiply(ntc_gf256_engine* e, uint32_t w, const uint8_t* src, uint8_t* dst,
                           size_t len, uint32_t c, int add, void* stream)
{
  if (!e || (len && (!src || !dst))) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (!valid_w(w)) return fail(NTC_GPU_EINVAL, "w must be 4, 8, 16 or 32");
  if (len == 0) return NTC_GPU_OK;
  const uint64_t blocks = (len / 4 + 1 + 255) / 256;
  if (blocks > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "region too large for one launch");
  (void)hipSetDevice(e->device);
  auto* fn = w == 4 ? gfw_region<4> : w == 8 ? gfw_region<8> : w == 16 ? gfw_region<16> : gfw_region<32>;
  hipLaunchKernelGGL(fn, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), src, dst, static_cast<uint64_t>(len), c, add);
  return hip_check(hipGetLastError(), "gfw_region launch");
}

}  // extern "C"
