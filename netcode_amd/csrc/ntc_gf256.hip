// ntc_gf256.hip -- MI355X (gfx950) GF(2^8) network-coding engine: kernels + C ABI.
//
// Hot path of ahamez/netcode: the region multiply-accumulate behind
// ntc::detail::encoder (netcode/detail/encoder.cc:15-64) and ntc::detail::decoder
// (netcode/detail/decoder.cc:393-408, 412-566), batched over independent generations.
//
// Kernels
//   encode_mac<R,D>     rep[g][row0..row0+R) = A_g * src[g] over one column slice; A_g's entries
//                       are the reference coefficients, computed in scalar registers.
//   decode_plan         one wave per generation: masks -> missing / received lists, greedy repair
//                       selection with device Gauss-Jordan (reference failure semantics), the
//                       m x k decode matrix D = [M^-1 | M^-1 * C_recv], decoded sizes, status.
//   decode_mac<R,D>     src[g][missing] = D_g * [repairs ; received sources] (same MAC core).
//   region_mul          dst = c*src / dst ^= c*src (galois_field::multiply / multiply_add).
//
// The MAC core: a wave owns a 64 x 4D-byte column slice of one generation; each lane keeps R x D
// dword accumulators.  c*x for four bytes at once = three v_perm_b32 table lookups (bits 0-2,
// 3-5, 6-7 of every byte) whose tables live in scalar registers; accumulation by v_bitop3_b32
// (3-input XOR).  Sources are processed in pairs: 6 v_perm + 3 v_bitop3 per dword pair.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>

#include "gf256_field.hh"
#include "engine.hh"
#include "netcode/gpu.h"

namespace ntcgpu {

__constant__ __attribute__((aligned(16))) PermTables d_perm = make_perm_tables();
__constant__ __attribute__((aligned(16))) FieldTables d_field = make_field_tables();

constexpr int kWaves = 4;               // waves per 256-thread block
constexpr int kMaxPlanRows = 64;        // r <= 64: wave-level plan kernels; larger r: decode_plan_big

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}

// Same op through the compiler builtin: schedulable, no inline-asm hazard padding.
__device__ __forceinline__ uint32_t bxor3(uint32_t a, uint32_t b, uint32_t c)
{
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

__device__ __forceinline__ uint32_t uniform(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

template <int D> struct RowVec;
template <> struct RowVec<1> { using T = uint32_t; };
template <> struct RowVec<2> { using T = uint2; };
template <> struct RowVec<4> { using T = uint4; };

template <int D>
__device__ __forceinline__ void load_row(const uint8_t* p, uint32_t (&x)[D])
{
  const typename RowVec<D>::T v = *reinterpret_cast<const typename RowVec<D>::T*>(p);
  if constexpr (D == 1) {
    x[0] = v;
  } else if constexpr (D == 2) {
    x[0] = v.x; x[1] = v.y;
  } else {
    x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
  }
}

template <int D>
__device__ __forceinline__ void store_row(uint8_t* p, const uint32_t (&x)[D])
{
  using T = typename RowVec<D>::T;
  T v;
  if constexpr (D == 1) {
    v = x[0];
  } else if constexpr (D == 2) {
    v.x = x[0]; v.y = x[1];
  } else {
    v.x = x[0]; v.y = x[1]; v.z = x[2]; v.w = x[3];
  }
  *reinterpret_cast<T*>(p) = v;
}

// Selectors for the three lookups of one source dword.
template <int D>
struct Sel {
  uint32_t a[D], b[D], e[D];
  __device__ __forceinline__ void make(const uint32_t (&x)[D])
  {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      a[d] = x[d] & 0x07070707u;
      b[d] = (x[d] >> 3) & 0x07070707u;
      e[d] = (x[d] >> 6) & 0x03030303u;
    }
  }
};

// acc ^= c0*x0 ^ c1*x1 for D dwords (two sources, one repair row).
template <int D>
__device__ __forceinline__ void mac2(uint32_t (&acc)[D], uint32_t c0, const Sel<D>& s0,
                                     uint32_t c1, const Sel<D>& s1)
{
  const uint32_t* t0 = d_perm.w[c0];
  const uint32_t* t1 = d_perm.w[c1];
  const uint32_t a00 = t0[0], a01 = t0[1], b00 = t0[2], b01 = t0[3], e0 = t0[4];
  const uint32_t a10 = t1[0], a11 = t1[1], b10 = t1[2], b11 = t1[3], e1 = t1[4];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint32_t p = xor3(__builtin_amdgcn_perm(a01, a00, s0.a[d]),
                            __builtin_amdgcn_perm(b01, b00, s0.b[d]),
                            __builtin_amdgcn_perm(e0, e0, s0.e[d]));
    const uint32_t q = xor3(__builtin_amdgcn_perm(a11, a10, s1.a[d]),
                            __builtin_amdgcn_perm(b11, b10, s1.b[d]),
                            __builtin_amdgcn_perm(e1, e1, s1.e[d]));
    acc[d] = xor3(acc[d], p, q);
  }
}

template <int D>
__device__ __forceinline__ void mac1(uint32_t (&acc)[D], uint32_t c0, const Sel<D>& s0)
{
  const uint32_t* t0 = d_perm.w[c0];
  const uint32_t a00 = t0[0], a01 = t0[1], b00 = t0[2], b01 = t0[3], e0 = t0[4];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    acc[d] = xor3(acc[d], __builtin_amdgcn_perm(a01, a00, s0.a[d]),
                  __builtin_amdgcn_perm(b01, b00, s0.b[d])) ^
             __builtin_amdgcn_perm(e0, e0, s0.e[d]);
  }
}

__device__ __forceinline__ uint8_t gmul(uint8_t a, uint8_t b)
{
  return (a == 0 || b == 0) ? 0 : d_field.exp[d_field.log[a] + d_field.log[b]];
}

__device__ __forceinline__ uint32_t field_inv_dev(uint32_t x)
{
  return d_field.exp[(255 - d_field.log[x]) % 255];
}

__device__ __forceinline__ uint16_t mul_size(uint16_t size, uint8_t c)
{
  // netcode/detail/galois_field.hh:108-115: a u16 coded as a 2-byte region.
  return static_cast<uint16_t>(gmul(c, static_cast<uint8_t>(size & 0xFF)) |
                               (gmul(c, static_cast<uint8_t>(size >> 8)) << 8));
}

struct MacArgs {
  uint32_t G, k, stride;
  uint32_t rows;               // encode: r; decode: r (the plan holds m <= r rows per generation)
  uint32_t nrowchunks, ncolchunks;
  const uint8_t* in0;          // [G][k][stride] sources (encode input / decode received slots)
  const uint8_t* in1;          // decode: repairs [G][rows][stride]
  uint8_t* out;                // encode: repairs [G][rows][stride]; decode: source slots (in place)
  const uint16_t* rows_per_gen;  // decode: plan_m [G]
  const uint16_t* in_idx;      // decode: plan_in [G][k] (< k: source slot, >= k: repair slot + k)
  const uint16_t* out_idx;     // decode: plan_out [G][rp] (destination source slot per row)
  const uint8_t* coef;         // [G][k][rp] coefficient bytes, row-minor
  uint32_t rp;
  const uint64_t* row_ptr;     // bit-sliced decode: input row address per plan position,
                               // [G][k + kBsRing] (plan_rows; the tail repeats position k-1)
  uint32_t tile_fast;          // bit-sliced task order: 1 = row tile fastest, 0 = column span fastest
  const uint8_t* pair;         // encode pairing flags [G] (gf_mac_bs<.., PAIR>), see kPairGap
  uint64_t pair_in, pair_out;  // byte distance of the partner's sources / repairs
  // split-k (bit-sliced encode / combine with less than one round of tasks): part ks sums the
  // sources [ks * kpart, (ks + 1) * kpart) into out (ks = 0) or kout + (ks - 1) * kout_step, and
  // ksplit_reduce folds the parts into out
  uint32_t ksplit, kpart;
  uint8_t* kout;
  uint64_t kout_step;
};

// ---- hand-scheduled scalar loads -------------------------------------------------------------
// The per-row lookup tables and the coefficient words are wave-uniform; they travel through the
// scalar cache into SGPRs.  hipcc schedules those loads lazily (load -> s_waitcnt lgkmcnt(0) ->
// use, one round trip per few rows), so they are issued here by inline asm one row (tables) or
// one source pair (coefficient words) ahead.  SMEM returns out of order, so every wait is
// lgkmcnt(0); the "+s" operands tie each consumer to the wait that retires its load.
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

struct Tab {
  u32x4 ab;   // {a_lo, a_hi, b_lo, b_hi}
  uint32_t e;
};

__device__ __forceinline__ Tab sload_table(uint32_t c)
{
  Tab t;
  asm volatile("s_load_dwordx4 %0, %2, %3\n\ts_load_dword %1, %2, %3 offset:0x10"
               : "=&s"(t.ab), "=s"(t.e) : "s"(&d_perm.w[0][0]), "s"(c << 5) : "memory");
  return t;
}

template <int NW> struct CW;
template <> struct CW<1> { using T = uint32_t; };
template <> struct CW<2> { using T = u32x2; };
template <> struct CW<4> { using T = u32x4; };
template <> struct CW<8> { using T = u32x8; };

template <int NW>
__device__ __forceinline__ typename CW<NW>::T sload_words(const uint8_t* p)
{
  typename CW<NW>::T v;
  if constexpr (NW == 1) asm volatile("s_load_dword %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
  else if constexpr (NW == 2) asm volatile("s_load_dwordx2 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
  else if constexpr (NW == 4) asm volatile("s_load_dwordx4 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
  else asm volatile("s_load_dwordx8 %0, %1, 0x0" : "=s"(v) : "s"(p) : "memory");
  return v;
}

template <int NW>
__device__ __forceinline__ uint32_t cbyte(const typename CW<NW>::T& w, int j)
{
  uint32_t word;
  if constexpr (NW == 1) word = w;
  else word = w[j >> 2];
  return (word >> (8 * (j & 3))) & 0xFFu;
}

template <int D>
__device__ __forceinline__ void mac2t(uint32_t (&acc)[D], const Tab& t0, const Sel<D>& s0,
                                      const Tab& t1, const Sel<D>& s1)
{
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const uint32_t p = xor3(__builtin_amdgcn_perm(t0.ab[1], t0.ab[0], s0.a[d]),
                            __builtin_amdgcn_perm(t0.ab[3], t0.ab[2], s0.b[d]),
                            __builtin_amdgcn_perm(t0.e, t0.e, s0.e[d]));
    const uint32_t q = xor3(__builtin_amdgcn_perm(t1.ab[1], t1.ab[0], s1.a[d]),
                            __builtin_amdgcn_perm(t1.ab[3], t1.ab[2], s1.b[d]),
                            __builtin_amdgcn_perm(t1.e, t1.e, s1.e[d]));
    acc[d] = xor3(acc[d], p, q);
  }
}

// One wave computes R output rows x (64 lanes x 4D bytes) of one generation:
//   out[row] = sum_i coef[i][row] * in[i]
// Inputs are consumed in pairs with the next pair's loads in flight (register double buffer).
template <int R, int D, bool DEC>
__device__ __forceinline__ void mac_tile(const MacArgs& a, uint32_t g, uint32_t row0, uint32_t nrows,
                                         uint32_t col, bool active)
{
  constexpr int NW = R / 4;   // coefficient words per input for this row tile
  using CWT = typename CW<NW>::T;
  const size_t stride = a.stride;
  const uint32_t k = a.k;
  const uint32_t colx = active ? col : 0u;
  const uint8_t* base0 = a.in0 + static_cast<size_t>(g) * k * stride + colx;
  const uint8_t* base1 = DEC ? a.in1 + static_cast<size_t>(g) * a.rows * stride + colx : nullptr;
  const uint16_t* in = DEC ? a.in_idx + static_cast<size_t>(g) * k : nullptr;
  const uint8_t* coef = a.coef + static_cast<size_t>(g) * k * a.rp + row0;
  const uint32_t rp = a.rp;
  auto rowptr = [&](uint32_t i) -> const uint8_t* {
    if constexpr (DEC) {
      const uint32_t ii = uniform(in[i]);
      return ii < k ? base0 + ii * stride : base1 + (ii - k) * stride;
    } else {
      return base0 + i * stride;
    }
  };

  uint32_t acc[R][D];
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int d = 0; d < D; ++d) acc[j][d] = 0;

  const uint32_t kk = k & ~1u;
  if (kk) {
    uint32_t n0[D], n1[D];
    load_row<D>(rowptr(0), n0);
    load_row<D>(rowptr(1), n1);
    CWT w0 = sload_words<NW>(coef);
    CWT w1 = sload_words<NW>(coef + rp);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(w0), "+s"(w1) :: "memory");
    Tab t0 = sload_table(cbyte<NW>(w0, 0));
    Tab t1 = sload_table(cbyte<NW>(w1, 0));
    for (uint32_t i = 0; i < kk; i += 2) {
      uint32_t x0[D], x1[D];
#pragma unroll
      for (int d = 0; d < D; ++d) { x0[d] = n0[d]; x1[d] = n1[d]; }
      const bool more = i + 2 < kk;
      if (more) {
        load_row<D>(rowptr(i + 2), n0);
        load_row<D>(rowptr(i + 3), n1);
      }
      Sel<D> s0, s1;
      s0.make(x0);
      s1.make(x1);
      CWT nw0 = w0, nw1 = w1;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        // retire row j's tables (issued one row earlier); then put row j+1's in flight
        if (j == R - 1) {
          asm volatile("s_waitcnt lgkmcnt(0)"
                       : "+s"(t0.ab), "+s"(t0.e), "+s"(t1.ab), "+s"(t1.e), "+s"(nw0), "+s"(nw1) :: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(t0.ab), "+s"(t0.e), "+s"(t1.ab), "+s"(t1.e) :: "memory");
        }
        if (j == 0 && more) {
          nw0 = sload_words<NW>(coef + (i + 2) * rp);
          nw1 = sload_words<NW>(coef + (i + 3) * rp);
        }
        Tab u0, u1;
        if (j + 1 < R) {
          u0 = sload_table(cbyte<NW>(w0, j + 1));
          u1 = sload_table(cbyte<NW>(w1, j + 1));
        } else if (more) {
          u0 = sload_table(cbyte<NW>(nw0, 0));
          u1 = sload_table(cbyte<NW>(nw1, 0));
        } else {
          u0 = t0;
          u1 = t1;
        }
        mac2t<D>(acc[j], t0, s0, t1, s1);
        t0 = u0;
        t1 = u1;
      }
      w0 = nw0;
      w1 = nw1;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (k & 1u) {
    uint32_t x0[D];
    load_row<D>(rowptr(kk), x0);
    Sel<D> s0;
    s0.make(x0);
    const uint32_t* cw0 = reinterpret_cast<const uint32_t*>(coef + kk * rp);
#pragma unroll
    for (int j = 0; j < R; ++j) mac1<D>(acc[j], (cw0[j >> 2] >> (8 * (j & 3))) & 0xFFu, s0);
  }

  if (!active) return;
  if constexpr (DEC) {
    const uint16_t* outs = a.out_idx + static_cast<size_t>(g) * a.rp + row0;
    uint8_t* base = a.out + static_cast<size_t>(g) * k * stride + col;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (static_cast<uint32_t>(j) < nrows) store_row<D>(base + uniform(outs[j]) * stride, acc[j]);
  } else {
    uint8_t* base = a.out + (static_cast<size_t>(g) * a.rows + row0) * stride + col;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (static_cast<uint32_t>(j) < nrows) store_row<D>(base + j * stride, acc[j]);
  }
}

// ---- bit-sliced MAC ------------------------------------------------------------------------
// A lane owns 32 bytes = 8 dwords of a 2 KiB column span.  transpose8 turns them into 8 bit-
// planes (plane p = bit p of every byte; an involution, so the same code slices and un-slices).
// Multiplication by c is then linear over GF(2): plane p of c*x is an XOR of input planes.  Per
// source the XOR combinations of planes 0-3 and of planes 4-7 are built once (Four-Russians
// tables, 30 planes, NTC_BS_TABLES) and the tile's rows run as a chain of jumps into one shared
// table of 256 blocks, block c = the <= 8 v_bitop3 of acc ^= c*x on the row selected by VGPR-
// relative addressing (gf_bitslice_table.inc, tools/gen_bitslice_table.py).
#include "gf_bitslice_table.inc"

// The block table, once per code object: never called (it starts with s_endpgm); the MAC kernels
// enter it with s_swappc and it returns through s92:93.
extern "C" __device__ __attribute__((used, noinline)) void ntc_bs_tables() { asm volatile(NTC_BS_TABLE_ASM); }

// Delta swap of the `mask` bit groups of b with the groups `sh` bits higher in a: two shifts and
// two bit-field inserts (v_bitop3 select), 4 VALU.
__device__ __forceinline__ void swap_blocks(uint32_t& a, uint32_t& b, uint32_t sh, uint32_t mask)
{
  // bitop3 0xCA = S0 ? S1 : S2 (bitwise select)
  const uint32_t na = __builtin_amdgcn_bitop3_b32(mask << sh, b << sh, a, 0xCA);
  const uint32_t nb = __builtin_amdgcn_bitop3_b32(mask, a >> sh, b, 0xCA);
  a = na;
  b = nb;
}

// The delta-swap constants in VGPRs.  On gfx950 a VALU op issues at half rate when it reads an
// SGPR (any slot) or has a constant in src0 (tools/gen_mb_issue.py, profiles/r05/mb_issue*.log:
// v_bitop3 / v_xor with an SGPR, v_lshlrev_b32 with an inline-constant shift amount, v_alignbit,
// v_lshl_or, v_bfi, v_lshlrev_b64: 4.2-4.9 cycles per SIMD; VGPR-only v_bitop3 / v_xor / v_add /
// v_lshrrev with a VGPR amount: 2.3).  The compiler keeps constants in SGPRs and shift amounts as
// inline constants, which would halve the transpose's rate; these come out of an asm statement,
// so they stay in VGPRs.
struct TMasks {
  uint32_t m4, m2, m1;                     // 0x0F0F0F0F, 0x33333333, 0x55555555
  uint32_t s4, s2, s1;                     // shift amounts 4, 2, 1
};

template <bool VSH = true>
__device__ __forceinline__ TMasks tmasks()
{
  TMasks t;
  asm volatile("v_mov_b32 %0, 0x0f0f0f0f\n\tv_mov_b32 %1, 0x33333333\n\tv_mov_b32 %2, 0x55555555"
               : "=v"(t.m4), "=v"(t.m2), "=v"(t.m1));
  if constexpr (VSH)
    asm volatile("v_mov_b32 %0, 4\n\tv_mov_b32 %1, 2\n\tv_mov_b32 %2, 1" : "=v"(t.s4), "=v"(t.s2), "=v"(t.s1));
  else
    t.s4 = 4, t.s2 = 2, t.s1 = 1;
  return t;
}

// swap_blocks with VGPR operands only: m = ~(m << sh) for the three masks, so both selects use m
__device__ __forceinline__ void swap_m(uint32_t& a, uint32_t& b, uint32_t sh, uint32_t m)
{
  const uint32_t na = __builtin_amdgcn_bitop3_b32(m, a, b << sh, 0xCA);     // m ? a : b << sh
  const uint32_t nb = __builtin_amdgcn_bitop3_b32(m, a >> sh, b, 0xCA);     // m ? a >> sh : b
  a = na;
  b = nb;
}

template <bool VSH = true>
__device__ __forceinline__ void transpose8(uint32_t* d, const TMasks& t)
{
#pragma unroll
  for (int i = 0; i < 4; ++i) swap_m(d[i], d[i + 4], VSH ? t.s4 : 4u, t.m4);
#pragma unroll
  for (int i = 0; i < 8; i += 4) {
    swap_m(d[i], d[i + 2], VSH ? t.s2 : 2u, t.m2);
    swap_m(d[i + 1], d[i + 3], VSH ? t.s2 : 2u, t.m2);
  }
#pragma unroll
  for (int i = 0; i < 8; i += 2) swap_m(d[i], d[i + 1], VSH ? t.s1 : 1u, t.m1);
}

__device__ __forceinline__ void transpose8(uint32_t* d)
{
#pragma unroll
  for (int i = 0; i < 4; ++i) swap_blocks(d[i], d[i + 4], 4, 0x0F0F0F0Fu);
#pragma unroll
  for (int i = 0; i < 8; i += 4) {
    swap_blocks(d[i], d[i + 2], 2, 0x33333333u);
    swap_blocks(d[i + 1], d[i + 3], 2, 0x33333333u);
  }
#pragma unroll
  for (int i = 0; i < 8; i += 2) swap_blocks(d[i], d[i + 1], 1, 0x55555555u);
}

// Loads through the constant address space: always scalar (s_load) for a uniform address, with
// the waits placed by the compiler.  Used for data no kernel in flight writes (coefficients,
// plans, row addresses).
template <typename T>
__device__ __forceinline__ T const_load(const void* p)
{
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(
      reinterpret_cast<uintptr_t>(p));
}

// A u16 of a device array through the scalar unit (the aligned dword around it): a decode MAC
// wave's row count comes from the plan this way, beside the kernel arguments, instead of through
// a vector load whose whole memory round trip preceded everything else the wave issued.
__device__ __forceinline__ uint32_t const_load_u16(const uint16_t* p)
{
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t w = const_load<uint32_t>(reinterpret_cast<const void*>(a & ~static_cast<uintptr_t>(3)));
  return (w >> (8u * static_cast<uint32_t>(a & 2u))) & 0xFFFFu;
}

// Source staging: every wave streams its sources through a private ring of kBsRing LDS slots with
// LDS-DMA (global_load_lds_dwordx4), kBsRing-1 sources ahead, so HBM latency hides behind ~3
// chain iterations without holding VGPRs.  A lane owns two 16-byte pieces of the 2 KiB column
// span -- bytes [16*lane, +16) and [1024 + 16*lane, +16) -- so each DMA and each store is one
// contiguous KiB per wave, and a piece is valid whenever its 16 bytes lie inside the stride.
constexpr int kBsRing = 4;              // LDS slots per wave (the loop is unrolled by it)
constexpr uint32_t kBsSlot = 2048;      // one source's column span
constexpr int kBsWaves = 4;             // waves (independent tasks) per workgroup

__device__ __forceinline__ uint32_t lds_addr(const void* p)
{
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(
          reinterpret_cast<uintptr_t>(p))));
}

// Wait until at most N of this wave's vector-memory operations (LDS-DMA included) are in flight.
// The "memory" clobber keeps the LDS reads of the slot below the wait.
template <int N>
__device__ __forceinline__ void vm_wait()
{
  asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory");
}

// The block table's address: the fast copy, or the safe one if the fast copy straddles a 4 GiB
// boundary.  The table sits anywhere in the code object, so the PC-relative offset is a signed
// 64-bit quantity, added as low half + high half with carry (s_getpc returns the s_add's address;
// the lo literal sits 4 bytes after it, the hi literal 12).
__device__ __forceinline__ uint64_t bs_table_base()
{
  uint64_t tb;
  asm volatile("s_getpc_b64 s[96:97]\n"
               "s_add_u32 s96, s96, ntc_bs_f@rel32@lo+4\n"
               "s_addc_u32 s97, s97, ntc_bs_f@rel32@hi+12\n"
               "s_add_u32 s98, s96, %1\n"
               "s_cbranch_scc0 LBSo%=\n"
               "s_getpc_b64 s[96:97]\n"
               "s_add_u32 s96, s96, ntc_bs_s@rel32@lo+4\n"
               "s_addc_u32 s97, s97, ntc_bs_s@rel32@hi+12\n"
               "LBSo%=:\n"
               "s_mov_b64 %0, s[96:97]\n"
               : "=s"(tb) : "i"(kBsSpan + 64) : "s96", "s97", "s98", "scc");
  return tb;
}

template <int R> struct BsCoef;
template <> struct BsCoef<8> { using T = u32x2; };
template <> struct BsCoef<16> { using T = u32x4; };

// One wave: rows [tile*R, tile*R + nrows) of generation g over the 2 KiB column span cc.
//   encode: out[row] = sum_i coef[g][i][row] * in0[g][i]
//   decode: out[out_idx[row]] = sum_i plan_coef[g][i][row] * (input row i of the plan)
// R = 8: accumulators v32..v95 (<= 128 VGPRs, 4 waves per SIMD).  R = 16: v32..v159, the
// source's transpose and plane tables amortised over twice the rows, <= 168 VGPRs (3 waves per
// SIMD); its source is read from LDS at the top of its own iteration (no register copy of the
// next one).  FULL: the span lies inside the stride (stride % 2048 == 0), so both pieces come
// from one lane offset; else each piece has its own, clamped to the span's first bytes when it
// lies past the stride (loaded, never stored).  PAIR (encode, stride <= 1024): the second piece
// of each lane holds the same bytes of the partner generation (poff_in / poff_out bytes further
// on; 0 and never stored when the generation is alone).  SL (encode / combine, FULL): in0 holds
// the sources already bit-sliced by bs_preslice, so the fill is the plane tables alone.
template <int R, bool DEC, bool FULL, bool PAIR = false, bool SL = false>
__device__ __forceinline__ void bs_tile(const MacArgs& a, uint32_t g, uint32_t tile,
                                        uint32_t nrows, uint32_t cc, uint32_t lane, uint32_t ring,
                                        uint64_t poff_in = 0, uint64_t poff_out = 0,
                                        uint32_t i_begin = 0, uint32_t i_count = 0,
                                        uint8_t* out_base = nullptr)
{
  static_assert(R == 8 || R == 16, "8- or 16-row tiles");
  static_assert(!PAIR || (!DEC && !FULL), "pairing is an encode mode for short symbols");
  static_assert(!SL || (!DEC && FULL && !PAIR), "pre-sliced sources: whole spans of an encode / combine");
  static_assert(kBsRing == 4, "the unrolled loop assumes a 4-slot ring");
#ifdef NTC_ABL_KLATE       // timing-only experiment builds: the late source read for every 16-row tile
  constexpr bool kLate = R == 16;
#else
  constexpr bool kLate = R == 16 && !FULL;
#endif
  using CoefV = typename BsCoef<R>::T;
  const size_t stride = a.stride;
  const uint32_t k = i_count ? i_count : a.k;           // sources this wave sums (split-k: a part)
  const uint32_t col = cc * 2048u;
  // One VGPR serves the LDS reads and the (FULL) DMA offsets: x = ring + 16*lane; the DMA's
  // scalar row base is pre-biased by col - ring.
  const uint32_t x = ring + lane * 16u;
  const bool v0 = FULL || col + lane * 16u < stride;
  const bool v1 = PAIR ? poff_out != 0 && v0 : FULL || col + lane * 16u + 1024u < stride;
  const uint32_t d0 = v0 ? x : ring, d1 = v1 ? (PAIR ? x : x + 1024u) : ring;   // !FULL DMA offsets
  const uint8_t* base0 = a.in0 + (static_cast<size_t>(g) * a.k + i_begin) * stride;
  const uint64_t* rowp = DEC ? a.row_ptr + static_cast<size_t>(g) * (a.k + kBsRing) : nullptr;
  const uint32_t jstep = a.rp;
  const uint8_t* jp = a.coef + (static_cast<size_t>(g) * a.k + i_begin) * a.rp + tile * R;
  const uint64_t bias = static_cast<uint64_t>(col) - ring;
  auto row_at = [&](uint32_t i) -> const uint8_t* {    // a scalar (SGPR) row address
    uint64_t v;
    if constexpr (DEC) v = const_load<uint64_t>(rowp + i);
    else v = reinterpret_cast<uint64_t>(base0 + (i < k ? i : k - 1) * stride);
    const uint32_t lo = uniform(static_cast<uint32_t>(v)), hi = uniform(static_cast<uint32_t>(v >> 32));
    return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  auto lds_row = [&](uint32_t slot, uint32_t (&y)[8]) {
    const auto* p = reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(x + slot * kBsSlot);
    const u32x4 q0 = p[0], q1 = p[1024 / 16];
    y[0] = q0[0]; y[1] = q0[1]; y[2] = q0[2]; y[3] = q0[3];
    y[4] = q1[0]; y[5] = q1[1]; y[6] = q1[2]; y[7] = q1[3];
  };
  // prologue DMAs (slots 0 .. kBsRing-2): the same instructions as the loop's refill
  auto dma = [&](const uint8_t* row, uint32_t slot) {
    uint32_t keep;
    if constexpr (FULL)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, %2\n\t"
                   "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(x), "s"(row), "s"(slot) : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, %3\n\t"
                   "s_add_u32 m0, %4, 0x400\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %2, %5\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(d0), "v"(d1), "s"(row), "s"(slot), "s"(row + (PAIR ? poff_in : 0))
                   : "memory", "scc");
  };

  u32x8 A[R];
#pragma unroll
  for (int j = 0; j < R; ++j) A[j] = u32x8{0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t tbase = bs_table_base();
  uint32_t slotm[kBsRing];                             // M0 of each slot (loop-invariant SGPRs)
#pragma unroll
  for (int q = 0; q < kBsRing; ++q) slotm[q] = uniform(ring + q * kBsSlot);

#pragma unroll
  for (int q = 0; q < kBsRing - 1; ++q) dma(row_at(q) + bias, slotm[q]);
  const uint8_t* nrow = row_at(kBsRing - 1);           // the refill of iteration 0
  CoefV on = const_load<CoefV>(jp);
  uint32_t ycur[8];
  if constexpr (!kLate) {
    vm_wait<2 * (kBsRing - 2)>();
    lds_row(0, ycur);
  }
  for (uint32_t i0 = 0; i0 < k; i0 += kBsRing) {
#pragma unroll
    for (int u = 0; u < kBsRing; ++u) {
      const uint32_t i = i0 + u;
      if (i >= k) break;                               // uniform: k % 4 != 0
      const CoefV o = on;
      uint32_t Y[kBsPlanes];
      if constexpr (kLate) {
        vm_wait<2 * (kBsRing - 2)>();                  // source i has landed
        lds_row(u, ycur);
      }
#pragma unroll
      for (int p = 0; p < 8; ++p) Y[p] = ycur[p];
#ifndef NTC_ABL_NOFILL     // timing-only ablation builds (tools/build_variant.sh -DNTC_ABL_...)
      if constexpr (!SL) transpose8(Y);                // SL: bs_preslice already sliced the source
#endif
#ifdef NTC_ABL_FILL2       // timing-only: a second transpose of the same source, results discarded
      {
        uint32_t salt = 0, Z[8];
        asm volatile("" : "+v"(salt));
#pragma unroll
        for (int p = 0; p < 8; ++p) Z[p] = ycur[p] ^ salt;
#ifdef NTC_ABL_FILL2_VGPR  // the extra transpose with register masks and shift amounts
        transpose8<true>(Z, tmasks<true>());
#else
        transpose8(Z);
#endif
#pragma unroll
        for (int p = 0; p < 8; ++p) asm volatile("" :: "v"(Z[p]));
      }
#endif
      if constexpr (!kLate) {
        vm_wait<2 * (kBsRing - 3)>();                  // source i+1 has landed
        lds_row((u + 1) % kBsRing, ycur);
      }
      jp += (i + 1 < k) ? jstep : 0u;
      on = const_load<CoefV>(jp);
#ifndef NTC_ABL_NOFILL
      NTC_BS_TABLES(Y)
#else
#pragma unroll
      for (int p = 8; p < kBsPlanes; ++p) Y[p] = ycur[p & 7];
#endif
      uint64_t P0 = (static_cast<uint64_t>(o[1]) << 32) | o[0];
      const uint32_t slot = slotm[(u + kBsRing - 1) % kBsRing];
      // the DMA's biased row base, formed here (the scalar load of the row address was issued an
      // iteration ago, and this block's LDS wait already covered it); then the next refill's row
      // address, loaded before the chain so its latency hides behind it
      const uint8_t* row = nrow + bias;
      const uint8_t* row2 = PAIR ? row + poff_in : row;   // the second piece's row (pairing)
      const uint8_t* nrow_next = DEC ? row_at(i + kBsRing) : nrow + ((i + kBsRing < k) ? stride : 0u);
      // refill the slot of source i-1 with source i+3, then the chain (one M0 save / restore)
#ifndef NTC_ABL_NODMA
#define NTC_BS_DMA_FULL \
      "s_mov_b32 s94, m0\n" "s_mov_b32 m0, %[slot]\n" "s_nop 0\n" \
      "global_load_lds_dwordx4 %[x], %[row]\n" "global_load_lds_dwordx4 %[x], %[row] offset:1024\n"
#else                      // timing-only ablation: the ring keeps whatever it holds
#define NTC_BS_DMA_FULL "s_mov_b32 s94, m0\n"
#endif
#define NTC_BS_DMA_PART \
      "s_mov_b32 s94, m0\n" "s_mov_b32 m0, %[slot]\n" "s_nop 0\n" \
      "global_load_lds_dwordx4 %[d0], %[row]\n" "s_add_u32 m0, %[slot], 0x400\n" "s_nop 0\n" \
      "global_load_lds_dwordx4 %[d1], %[row2]\n"
#define NTC_BS_ENTER \
      "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)\n" \
      "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 17\n" \
      "s_add_u32 s98, s96, s98\n" "s_addc_u32 s99, s97, 0\n" \
      "s_swappc_b64 s[92:93], s[98:99]\n"
#ifdef NTC_ABL_NOCHAIN
#undef NTC_BS_ENTER
#define NTC_BS_ENTER ""
#define NTC_BS_LEAVE "s_mov_b32 m0, s94\n"
#else
#define NTC_BS_LEAVE "s_set_gpr_idx_off\n" "s_mov_b32 m0, s94\n"
#endif
#define NTC_BS_CLOB "s92", "s93", "s94", "s98", "s99", "scc", "memory"
      if constexpr (R == 8) {
        uint64_t Z = 0;                                // no second half (s[88:89], the table's stub)
        if constexpr (FULL)
          asm volatile(NTC_BS_DMA_FULL NTC_BS_ENTER NTC_BS_LEAVE
                       : NTC_BS_OUTS8(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(Z)
                       : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase), [slot] "s"(slot), [x] "v"(x),
                         [row] "s"(row)
                       : NTC_BS_CLOB);
        else
          asm volatile(NTC_BS_DMA_PART NTC_BS_ENTER NTC_BS_LEAVE
                       : NTC_BS_OUTS8(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(Z)
                       : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase), [slot] "s"(slot), [d0] "v"(d0),
                         [d1] "v"(d1), [row] "s"(row), [row2] "s"(row2)
                       : NTC_BS_CLOB);
      } else {
        uint64_t P1 = (static_cast<uint64_t>(o[3]) << 32) | o[2];     // rows 8-15: s[88:89]
        if constexpr (FULL)
          asm volatile(NTC_BS_DMA_FULL NTC_BS_ENTER NTC_BS_LEAVE
                       : NTC_BS_OUTS16(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(P1)
                       : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase), [slot] "s"(slot), [x] "v"(x),
                         [row] "s"(row)
                       : NTC_BS_CLOB);
        else
          asm volatile(NTC_BS_DMA_PART NTC_BS_ENTER NTC_BS_LEAVE
                       : NTC_BS_OUTS16(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(P1)
                       : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase), [slot] "s"(slot), [d0] "v"(d0),
                         [d1] "v"(d1), [row] "s"(row), [row2] "s"(row2)
                       : NTC_BS_CLOB);
      }
      nrow = nrow_next;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped trailing DMAs

  const uint32_t row0 = tile * R;
  const uint32_t c0 = col + lane * 16u, c1 = c0 + 1024u;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    if (static_cast<uint32_t>(j) >= nrows) continue;
    uint32_t acc[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = A[j][p];
    transpose8(acc);
    uint8_t* dst;
    if constexpr (DEC) {
      const uint16_t* outs = a.out_idx + static_cast<size_t>(g) * a.rp + row0;
      dst = a.out + static_cast<size_t>(g) * a.k * stride + uniform(outs[j]) * stride;
    } else {
      dst = (out_base ? out_base : a.out) + (static_cast<size_t>(g) * a.rows + row0 + j) * stride;
    }
    if (v0) *reinterpret_cast<uint4*>(dst + c0) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    if (v1) *reinterpret_cast<uint4*>(dst + (PAIR ? poff_out + c0 : c1)) = make_uint4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// One wave per (generation, R-row tile, 2 KiB column span).  Blocks are renumbered so that each
// XCD (block b runs on XCD b % 8) owns a contiguous range of tasks: the row tiles of one
// generation then share that XCD's L2 instead of each pulling the sources from HBM.
template <int R, bool DEC, bool FULL, bool PAIR = false, bool SL = false>
__global__ __launch_bounds__(64 * kBsWaves)
__attribute__((amdgpu_waves_per_eu(R == 16 ? 3 : 4))) void gf_mac_bs(MacArgs a)
{
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[kBsWaves * kBsRing * kBsSlot];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = uniform(threadIdx.x >> 6);
  const uint32_t nb = gridDim.x;                       // a multiple of 8 (launch_mac)
  const uint32_t b = (blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3);
  uint32_t task = uniform(b * kBsWaves + wave);
  // few generations (dense, G = 1): row tiles fastest, so an XCD owns whole column spans and its
  // L2 serves each source slice to every row tile; many generations: column spans fastest
  uint32_t cc, tile;
  if (a.tile_fast) {
    tile = task % a.nrowchunks;
    task /= a.nrowchunks;
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
  } else {
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
    tile = task % a.nrowchunks;
    task /= a.nrowchunks;
  }
  uint32_t ks = 0;
  if (!DEC && !PAIR && a.ksplit > 1) {
    ks = task % a.ksplit;
    task /= a.ksplit;
  }
  const uint32_t g = task;
  if (g >= a.G) return;
  const uint32_t total = DEC ? const_load_u16(a.rows_per_gen + g) : a.rows;
  const uint32_t row0 = tile * R;
  if (row0 >= total) return;
  const uint32_t nrows = min(static_cast<uint32_t>(R), total - row0);
  const uint32_t ring = lds_addr(s_ring + wave * (kBsRing * kBsSlot));
  if (!DEC && !PAIR && a.ksplit > 1) {
    const uint32_t i0 = ks * a.kpart;                  // launch_mac: every part is non-empty
    bs_tile<R, DEC, FULL, false, SL>(a, g, tile, nrows, cc, lane, ring, 0, 0, i0, min(a.kpart, a.k - i0),
                                     ks ? a.kout + (ks - 1) * a.kout_step : a.out);
  } else if constexpr (PAIR) {
    const uint32_t pf = uniform(static_cast<uint32_t>(a.pair[g]));
    if (pf == 2) return;                               // encoded by its partner's wave
    bs_tile<R, DEC, FULL, true>(a, g, tile, nrows, cc, lane, ring, pf ? a.pair_in : 0, pf ? a.pair_out : 0);
  } else {
    bs_tile<R, DEC, FULL, false, SL>(a, g, tile, nrows, cc, lane, ring);
  }
}

// ---- paired bit-sliced MAC: the two 16-row tiles of a (generation, span) share the transpose ----
// The 48-op 8x8 bit transpose of a source depends only on the source, yet every 16-row tile of a
// generation repeated it (≈ 17-19 of the ≈ 66 cycles per row and source).  Here a
// 2-wave workgroup holds tiles 2p and 2p+1 of one (generation, 2 KiB span).  Sources go in turns of
// TS = 2J; in turn T wave w owns sources T*TS + 2j + w (j < J): it LDS-DMAs them two turns ahead,
// transposes each from its raw slot, publishes the 8 planes in that same slot and runs its own
// chain on them at once; its partner reads those planes one turn later.  Each wave transposes half
// the sources and builds its own 22 plane tables (NTC_BS_TABLES) from all of them -- only the
// 8 planes cross LDS (2 KiB, the bytes the raw source already occupies), unlike gf_mac_bsg's 30.
// Per turn, one barrier, placed before the last partner step:
//   own(T,0) partner(T-1,0) ... own(T,J-1) | barrier, DMA turn T+NS-1 | partner(T-1,J-1)
// It certifies that both waves published turn T's planes (read in turn T+1) and both finished
// reading turn T-1's, whose slots then take turn T+NS-1's DMA: NS slot sets of TS slots.  XOR is
// order-free, so the two waves summing the sources in different orders changes no byte.  Every
// LDS read -- raw bytes of an own source, planes of a partner source -- is issued one step ahead,
// into the ycur registers, as in bs_tile.
template <int J, int NS, bool DEC, bool FULL, uint32_t w>
__device__ __forceinline__ void bs_pair(const MacArgs& a, uint32_t g, uint32_t tile, uint32_t nrows,
                                        uint32_t cc, uint32_t lane, uint32_t ring)
{
  // w (the wave of the pair) is a template argument: own and partner slots are then immediate
  // offsets from one address register
  constexpr uint32_t TS = 2 * J;                       // sources per turn
  constexpr uint32_t kSet = TS * kBsSlot;              // LDS bytes of one turn's slots
  const size_t stride = a.stride;
  const uint32_t k = a.k;
  const uint32_t col = cc * 2048u;
  const uint32_t x = ring + lane * 16u;
  const bool v0 = FULL || col + lane * 16u < stride;
  const bool v1 = FULL || col + lane * 16u + 1024u < stride;
  const uint8_t* base0 = a.in0 + static_cast<size_t>(g) * k * stride;
  const uint64_t* rowp = DEC ? a.row_ptr + static_cast<size_t>(g) * (k + kBsRing) : nullptr;
  const uint8_t* jp0 = a.coef + static_cast<size_t>(g) * k * a.rp + tile * 16u;
  const uint32_t rp = a.rp;
  const uint64_t bias = static_cast<uint64_t>(col) - ring;
  const uint32_t nT = (k + TS - 1) / TS;
  auto row_at = [&](uint32_t i) -> const uint8_t* {    // scalar row address of source min(i, k-1)
    i = i < k ? i : k - 1;
    uint64_t v;
    if constexpr (DEC) v = const_load<uint64_t>(rowp + i);
    else v = reinterpret_cast<uint64_t>(base0 + static_cast<size_t>(i) * stride);
    const uint32_t lo = uniform(static_cast<uint32_t>(v)), hi = uniform(static_cast<uint32_t>(v >> 32));
    return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  auto coef_at = [&](uint32_t i) __attribute__((always_inline)) {   // zero past k: the chain returns at once
    return i < k ? const_load<u32x4>(jp0 + static_cast<size_t>(i) * rp) : u32x4{0, 0, 0, 0};
  };
  static_assert(NS == 3 || NS == 4, "3 or 4 slot sets");
  auto set_of = [](uint32_t T) { return (T % NS) * kSet; };   // LDS offset of turn T's slots
  // x is kept in v0 at every LDS access: with 128 accumulators, 30 table planes and the 8 ycur
  // registers only v0 / v1 are left, and the allocator otherwise spills x to make room for the
  // transpose's temporaries
  auto xv0 = [&]() __attribute__((always_inline)) {
    uint32_t v = x;
    asm volatile("" : "+{v0}"(v));
    return v;
  };
  // this wave's J sources of turn T into their slots (sources past k: the last one again, so every
  // turn issues 2J DMAs and the vmcnt arithmetic below holds)
  auto issue_turn = [&](uint32_t T) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint8_t* row = row_at(T * TS + 2 * j + w) + bias;
      const uint32_t m0 = uniform(ring + set_of(T) + (2 * j + w) * kBsSlot);
      uint32_t keep;
      if constexpr (FULL) {
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, %2\n\t"
                     "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(x), "s"(row), "s"(m0) : "memory");
      } else {
        // clamped offsets (loaded, never stored), formed here from an opaque copy of x so that
        // they are not kept live across the loop
        const uint32_t xx = xv0();
        const uint32_t d0 = v0 ? xx : ring, d1 = v1 ? xx + 1024u : ring;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %1, %3\n\t"
                     "s_add_u32 m0, %4, 0x400\n\ts_nop 0\n\t"
                     "global_load_lds_dwordx4 %2, %3\n\t"
                     "s_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(d0), "v"(d1), "s"(row), "s"(m0) : "memory", "scc");
      }
    }
  };
  // before reading own source j of turn T': the DMAs issued after it are the turn's later own
  // sources and the turns after T' issued so far -- up to T' + NS - 2 (at most nT)
  auto wait_own = [&](int j, uint32_t Tp) __attribute__((always_inline)) {
    const uint32_t na = Tp + (NS - 2) <= nT ? NS - 2 : (Tp <= nT ? nT - Tp : 0u);
    const int base = 2 * (J - 1 - j);
    if (na == 0) { if (base == 0) vm_wait<0>(); else vm_wait<2>(); }
    else if (na == 1) { if (base == 0) vm_wait<2 * J>(); else vm_wait<2 + 2 * J>(); }
    else { if (base == 0) vm_wait<4 * J>(); else vm_wait<2 + 4 * J>(); }
  };
  auto lds_read = [&](uint32_t off, uint32_t (&y)[8]) __attribute__((always_inline)) {
    const auto* p = reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(xv0() + off);
    const u32x4 q0 = p[0], q1 = p[1024 / 16];
    y[0] = q0[0]; y[1] = q0[1]; y[2] = q0[2]; y[3] = q0[3];
    y[4] = q1[0]; y[5] = q1[1]; y[6] = q1[2]; y[7] = q1[3];
  };
  auto lds_write = [&](uint32_t off, const uint32_t* y) __attribute__((always_inline)) {
    auto* p = reinterpret_cast<__attribute__((address_space(3))) u32x4*>(xv0() + off);
    p[0] = u32x4{y[0], y[1], y[2], y[3]};
    p[1024 / 16] = u32x4{y[4], y[5], y[6], y[7]};
  };
#ifndef NTC_ABL_NOBARRIER
  auto barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
#else                      // timing-only ablation (wrong results): no synchronisation of the pair
  auto barrier = []() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); };
#endif

  u32x8 A[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) A[j] = u32x8{0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t tbase = bs_table_base();
  auto chain = [&](const u32x4& o, uint32_t (&Y)[kBsPlanes]) __attribute__((always_inline)) {
    uint64_t P0 = (static_cast<uint64_t>(o[1]) << 32) | o[0];
    uint64_t P1 = (static_cast<uint64_t>(o[3]) << 32) | o[2];      // rows 8-15: s[88:89]
    asm volatile("s_mov_b32 s94, m0\n" NTC_BS_ENTER NTC_BS_LEAVE
                 : NTC_BS_OUTS16(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(P1)
                 : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase)
                 : NTC_BS_CLOB);
  };

  uint32_t ycur[8];
  u32x4 on;
  // own step: ycur = the raw bytes -> transpose -> publish the planes at `wr` -> issue the next
  // step's read -> tables -> chain.  Partner step: ycur = the planes -> next read -> tables -> chain.
  auto own_step = [&](uint32_t wr, auto&& next) __attribute__((always_inline)) {
    const u32x4 o = on;
    uint32_t Y[kBsPlanes];
#pragma unroll
    for (int p = 0; p < 8; ++p) Y[p] = ycur[p];
    transpose8(Y);
    lds_write(wr, Y);
    asm volatile("" ::: "memory");                     // the next read stays below the transpose
    next();
    NTC_BS_TABLES(Y)
    chain(o, Y);
  };
  auto partner_step = [&](auto&& next) __attribute__((always_inline)) {
    const u32x4 o = on;
    uint32_t Y[kBsPlanes];
    // a real copy (early-clobber asm), so that the allocator does not give ycur the table
    // registers v2..v9, which are live while the next read lands in ycur
#pragma unroll
    for (int p = 0; p < 8; ++p) asm volatile("v_mov_b32 %0, %1" : "=&v"(Y[p]) : "v"(ycur[p]));
    next();
    NTC_BS_TABLES(Y)
    chain(o, Y);
  };

  // Turns 0 .. nT, where turn nT's own sources are all past k: its own steps transpose the clamped
  // last source with zero coefficients (the chain returns at once) and exist only so that every
  // turn has the same steps -- the partner's last sources need no separate tail, and no step's
  // next read depends on a branch.
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) issue_turn(t);     // turns 0 .. NS-2 (past nT: clamped rows)
  wait_own(0, 0);
  lds_read(w * kBsSlot, ycur);
  on = coef_at(w);
  // turn 0: own steps only
#pragma unroll
  for (int j = 0; j < J; ++j)
    own_step((2 * j + w) * kBsSlot, [&]() __attribute__((always_inline)) {
      if (j + 1 < J) {
        wait_own(j + 1, 0);
        lds_read((2 * j + 2 + w) * kBsSlot, ycur);
        on = coef_at(2 * j + 2 + w);
      }
    });
  barrier();
  if (NS - 1 <= nT) issue_turn(NS - 1);
  wait_own(0, 1);                                      // next: own(1, 0)
  lds_read(kSet + w * kBsSlot, ycur);
  on = coef_at(TS + w);
  // turns 1 .. nT: own(T, j) then partner(T-1, j); S = T % NS at compile time, so the LDS offsets
  // are immediates
  auto turn = [&](uint32_t T, auto S) __attribute__((always_inline)) {
    constexpr uint32_t so = S() * kSet, sn = (S() + 1) % NS * kSet, sp = (S() + NS - 1) % NS * kSet;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      own_step(so + (2 * j + w) * kBsSlot, [&]() __attribute__((always_inline)) {
        lds_read(sp + (2 * j + 1 - w) * kBsSlot, ycur);    // partner(T-1, j), published last turn
        on = coef_at((T - 1) * TS + 2 * j + 1 - w);
      });
      if (j == J - 1) {
        barrier();
        if (T + NS - 1 <= nT) issue_turn(T + NS - 1);
      }
      partner_step([&]() __attribute__((always_inline)) {
        if (j + 1 < J) {                               // own(T, j+1)
          wait_own(j + 1, T);
          lds_read(so + (2 * j + 2 + w) * kBsSlot, ycur);
          on = coef_at(T * TS + 2 * j + 2 + w);
        } else {                                       // own(T+1, 0) (after turn nT: read, unused)
          wait_own(0, T + 1);
          lds_read(sn + w * kBsSlot, ycur);
          on = coef_at((T + 1) * TS + w);
        }
      });
    }
  };
  for (uint32_t T = 1; T <= nT; T += NS) {
    turn(T, std::integral_constant<uint32_t, 1>());
    if (T + 1 > nT) break;
    turn(T + 1, std::integral_constant<uint32_t, 2>());
    if (T + 2 > nT) break;
    if constexpr (NS == 4) {
      turn(T + 2, std::integral_constant<uint32_t, 3>());
      if (T + 3 > nT) break;
    }
    turn(T + NS - 1, std::integral_constant<uint32_t, 0>());
  }

  const uint32_t row0 = tile * 16u;
  const uint32_t c0 = col + lane * 16u, c1 = c0 + 1024u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (static_cast<uint32_t>(j) >= nrows) continue;
    uint32_t acc[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = A[j][p];
    transpose8(acc);
    uint8_t* dst;
    if constexpr (DEC) {
      const uint16_t* outs = a.out_idx + static_cast<size_t>(g) * a.rp + row0;
      dst = a.out + static_cast<size_t>(g) * a.k * stride + uniform(outs[j]) * stride;
    } else {
      dst = a.out + (static_cast<size_t>(g) * a.rows + row0 + j) * stride;
    }
    if (v0) *reinterpret_cast<uint4*>(dst + c0) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    if (v1) *reinterpret_cast<uint4*>(dst + c1) = make_uint4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// One 2-wave workgroup per (generation, pair of 16-row tiles, 2 KiB column span), blocks renumbered
// per XCD as in gf_mac_bs.  A pair whose second tile has no rows (a decode generation with m <= 16,
// the last tile of an odd tile count) runs gf_mac_bs's single-wave tile instead.
template <int J, int NS, bool DEC, bool FULL>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3))) void gf_mac_bsp(MacArgs a)
{
  static_assert(NS * 2 * J >= kBsRing, "the single-tile path uses a kBsRing-slot ring");
  __shared__ __attribute__((aligned(16))) uint8_t s_ring[NS * 2 * J * kBsSlot];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = uniform(threadIdx.x >> 6);
  const uint32_t nb = gridDim.x;                       // a multiple of 8 (launch_mac)
  uint32_t task = uniform((blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3));
  const uint32_t npair = (a.nrowchunks + 1) / 2;
  uint32_t cc, tp;
  if (a.tile_fast) {
    tp = task % npair;
    task /= npair;
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
  } else {
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
    tp = task % npair;
    task /= npair;
  }
  const uint32_t g = task;
  if (g >= a.G) return;
  const uint32_t total = DEC ? const_load_u16(a.rows_per_gen + g) : a.rows;
  const uint32_t row0 = tp * 32u;
  if (row0 >= total) return;
  const uint32_t ring = lds_addr(s_ring);
  if (total - row0 <= 16u) {                           // one tile: wave 0 alone
    if (w) return;
    bs_tile<16, DEC, FULL>(a, g, 2 * tp, total - row0, cc, lane, ring);
    return;
  }
  const uint32_t nrows = w ? min(16u, total - row0 - 16u) : 16u;
  if (w == 0) bs_pair<J, NS, DEC, FULL, 0>(a, g, 2 * tp, nrows, cc, lane, ring);
  else bs_pair<J, NS, DEC, FULL, 1>(a, g, 2 * tp + 1, nrows, cc, lane, ring);
}

// ---- grouped bit-sliced MAC: NT row tiles of one (generation, span) share the source fill ----
// The per-source fill -- the 8x8 bit transpose and the 22 plane-table XORs, 70+ VALU -- depends
// only on the source, not on the row tile, yet every 16-row tile of a generation repeated it.
// Here a workgroup holds the NT tiles of one (generation, 2 KiB column span): source i's 30 table
// planes are built ONCE, by wave i % NT, and published in LDS; every wave reads them (8 b128
// reads) and runs its own tile's chain.  Per source step:
//   read planes(i) from table slot i % 2 -> chain(i) -> [wave (i+1) % NT: build planes(i+1) into
//   slot (i+1) % 2] -> barrier
// Slot i % 2 is rewritten (with source i+2) only after the barrier that ends step i, when every
// wave has read it.  Each wave streams ITS OWN sources (s % NT == w) through a private ring of 2
// LDS slots by LDS-DMA, issued 2 * NT sources ahead, so no barrier guards the raw bytes.
// A wave whose tile has no rows (a decode generation with fewer rows than the group) still builds
// its share of the planes.
constexpr uint32_t kTabSlot = 8u * 1024u;   // 32 planes (30 used) x 64 lanes x 4 B, [quad][lane][4]
constexpr int kGrpRaw = 2;                  // raw-source slots per wave

template <int NT, bool DEC, bool FULL>
__device__ __forceinline__ void bs_group(const MacArgs& a, uint32_t g, uint32_t tile, uint32_t nrows,
                                         uint32_t cc, uint32_t lane, uint32_t w, uint32_t ring,
                                         uint32_t tabs, uint32_t i_begin, uint32_t i_count,
                                         uint32_t steps, bool idle, uint8_t* out_base)
{
  const size_t stride = a.stride;
  const uint32_t k = idle ? 0u : i_count;              // sources this group sums (<= steps)
  const uint32_t col = cc * 2048u;
  const uint32_t x = ring + lane * 16u;                 // LDS read offset of this lane's piece 0
  const bool v0 = FULL || col + lane * 16u < stride;
  const bool v1 = FULL || col + lane * 16u + 1024u < stride;
  const uint32_t d0 = v0 ? x : ring, d1 = v1 ? x + 1024u : ring;   // !FULL DMA offsets (clamped)
  const uint8_t* base0 = a.in0 + (static_cast<size_t>(g) * a.k + i_begin) * stride;
  const uint64_t* rowp = DEC ? a.row_ptr + static_cast<size_t>(g) * (a.k + kBsRing) : nullptr;
  const uint8_t* jp = a.coef + (static_cast<size_t>(g) * a.k + i_begin) * a.rp + tile * 16u;
  const uint64_t bias = static_cast<uint64_t>(col) - ring;
  const bool has_rows = nrows != 0;
  auto row_at = [&](uint32_t i) -> const uint8_t* {    // scalar row address of source i
    uint64_t v;
    if constexpr (DEC) v = const_load<uint64_t>(rowp + i);
    else v = reinterpret_cast<uint64_t>(base0 + static_cast<size_t>(i) * stride);
    const uint32_t lo = uniform(static_cast<uint32_t>(v)), hi = uniform(static_cast<uint32_t>(v >> 32));
    return reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(hi) << 32) | lo);
  };
  // raw slot of source s (this wave's s-th own source, s % NT == w): (s / NT) % 2
  auto dma = [&](uint32_t s) {
    const uint8_t* row = row_at(s) + bias;
    const uint32_t slot = uniform(ring + ((s / NT) & 1u) * kBsSlot);
    uint32_t keep;
    if constexpr (FULL)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, %2\n\t"
                   "global_load_lds_dwordx4 %1, %2 offset:1024\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(x), "s"(row), "s"(slot) : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %1, %3\n\t"
                   "s_add_u32 m0, %4, 0x400\n\ts_nop 0\n\t"
                   "global_load_lds_dwordx4 %2, %3\n\t"
                   "s_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(d0), "v"(d1), "s"(row), "s"(slot) : "memory", "scc");
  };
#ifndef NTC_GRP_VSH
#define NTC_GRP_VSH 0
#endif
  const TMasks tm = tmasks<NTC_GRP_VSH>();
  // build source s's planes (s % NT == w) from its raw slot into table slot s % 2
  auto produce = [&](uint32_t s) {
    if (s + NT < k) vm_wait<2>();                      // source s + NT is the younger DMA in flight
    else vm_wait<0>();
    const uint32_t slot = ((s / NT) & 1u) * kBsSlot;
    uint32_t Y[kBsPlanes];
    {
      const auto* p = reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(x + slot);
      const u32x4 q0 = p[0], q1 = p[1024 / 16];
      Y[0] = q0[0]; Y[1] = q0[1]; Y[2] = q0[2]; Y[3] = q0[3];
      Y[4] = q1[0]; Y[5] = q1[1]; Y[6] = q1[2]; Y[7] = q1[3];
    }
    // the slot's bytes are in registers once this wave's LDS reads return: refill it with the
    // wave's source two rounds on (the DMA writes LDS behind the reads, in issue order)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(Y[0]), "+v"(Y[1]), "+v"(Y[2]), "+v"(Y[3]), "+v"(Y[4]),
                 "+v"(Y[5]), "+v"(Y[6]), "+v"(Y[7]) :: "memory");
    if (s + 2 * NT < k) dma(s + 2 * NT);
    transpose8<NTC_GRP_VSH>(Y, tm);
    // planes published quad by quad as they are formed (NTC_BS_TABLES' order), so at most the
    // 8 input planes and one quad of combinations are live beside the accumulators
    auto* t = reinterpret_cast<__attribute__((address_space(3))) u32x4*>(tabs + (s & 1u) * kTabSlot + lane * 16u);
    t[0] = u32x4{Y[0], Y[1], Y[2], Y[3]};
    t[64] = u32x4{Y[4], Y[5], Y[6], Y[7]};
    Y[8] = Y[1] ^ Y[0]; Y[9] = Y[2] ^ Y[0]; Y[10] = Y[2] ^ Y[1]; Y[11] = Y[10] ^ Y[0];
    t[2 * 64] = u32x4{Y[8], Y[9], Y[10], Y[11]};
    Y[12] = Y[3] ^ Y[0]; Y[13] = Y[3] ^ Y[1]; Y[14] = Y[13] ^ Y[0]; Y[15] = Y[3] ^ Y[2];
    t[3 * 64] = u32x4{Y[12], Y[13], Y[14], Y[15]};
    Y[16] = Y[15] ^ Y[0]; Y[17] = Y[15] ^ Y[1]; Y[18] = Y[17] ^ Y[0]; Y[19] = Y[5] ^ Y[4];
    t[4 * 64] = u32x4{Y[16], Y[17], Y[18], Y[19]};
    Y[20] = Y[6] ^ Y[4]; Y[21] = Y[6] ^ Y[5]; Y[22] = Y[21] ^ Y[4]; Y[23] = Y[7] ^ Y[4];
    t[5 * 64] = u32x4{Y[20], Y[21], Y[22], Y[23]};
    Y[24] = Y[7] ^ Y[5]; Y[25] = Y[24] ^ Y[4]; Y[26] = Y[7] ^ Y[6]; Y[27] = Y[26] ^ Y[4];
    t[6 * 64] = u32x4{Y[24], Y[25], Y[26], Y[27]};
    Y[28] = Y[26] ^ Y[5]; Y[29] = Y[28] ^ Y[4];
    *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(&t[7 * 64]) = u32x2{Y[28], Y[29]};
  };
  static_assert(kBsPlanes == 30, "bs_group publishes the 30 planes of NTC_BS_TABLES");

  u32x8 A[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) A[j] = u32x8{0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t tbase = bs_table_base();
  // prologue: this wave's first two own sources in flight; wave 0 builds source 0
  if (w < k) dma(w);
  if (w + NT < k) dma(w + NT);
  if (w == 0 && k) produce(0);
  __syncthreads();
  u32x4 on = has_rows && k ? const_load<u32x4>(jp) : u32x4{0, 0, 0, 0};
  for (uint32_t i = 0; i < steps; ++i) {
    if (has_rows && i < k) {
      const u32x4 o = on;
      jp += a.rp;
      if (i + 1 < k) on = const_load<u32x4>(jp);
      uint32_t Y[kBsPlanes];
      {
        const auto* t = reinterpret_cast<const __attribute__((address_space(3))) u32x4*>(
            tabs + (i & 1u) * kTabSlot + lane * 16u);
#pragma unroll
        for (int q = 0; q < 7; ++q) {
          const u32x4 v = t[q * 64];
          Y[4 * q] = v[0]; Y[4 * q + 1] = v[1]; Y[4 * q + 2] = v[2]; Y[4 * q + 3] = v[3];
        }
        const u32x2 v = *reinterpret_cast<const __attribute__((address_space(3))) u32x2*>(&t[7 * 64]);
        Y[28] = v[0];
        Y[29] = v[1];
      }
      uint64_t P0 = (static_cast<uint64_t>(o[1]) << 32) | o[0];
      uint64_t P1 = (static_cast<uint64_t>(o[3]) << 32) | o[2];           // rows 8-15: s[88:89]
      asm volatile("s_mov_b32 s94, m0\n" NTC_BS_ENTER NTC_BS_LEAVE
                   : NTC_BS_OUTS16(A), [p] "+{s[90:91]}"(P0), [q] "+{s[88:89]}"(P1)
                   : NTC_BS_YPINS(Y), [tb] "{s[96:97]}"(tbase)
                   : NTC_BS_CLOB);
    }
    if (i + 1 < k && (i + 1) % NT == w) produce(i + 1);
    __syncthreads();
  }

  if (idle) return;
  const uint32_t row0 = tile * 16u;
  const uint32_t c0 = col + lane * 16u, c1 = c0 + 1024u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (static_cast<uint32_t>(j) >= nrows) continue;
    uint32_t acc[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) acc[p] = A[j][p];
    transpose8<NTC_GRP_VSH>(acc, tm);
    uint8_t* dst;
    if constexpr (DEC) {
      const uint16_t* outs = a.out_idx + static_cast<size_t>(g) * a.rp + row0;
      dst = a.out + static_cast<size_t>(g) * a.k * stride + uniform(outs[j]) * stride;
    } else {
      dst = out_base + (static_cast<size_t>(g) * a.rows + row0 + j) * stride;
    }
    if (v0) *reinterpret_cast<uint4*>(dst + c0) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
    if (v1) *reinterpret_cast<uint4*>(dst + c1) = make_uint4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// One workgroup of GPB groups of NT waves; group = (generation, NT 16-row tiles, 2 KiB column
// span[, split-k part]); blocks renumbered per XCD as in gf_mac_bs.  Four-wave workgroups (GPB =
// 2 pairs) are dispatched one wave per SIMD, like gf_mac_bs's; the groups share only the barrier.
template <int NT, bool DEC, bool FULL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void gf_mac_bsg(MacArgs a)
{
  constexpr uint32_t GPB = 4 / NT;
  __shared__ __attribute__((aligned(16))) uint8_t s_raw[GPB * NT * kGrpRaw * kBsSlot];
  __shared__ __attribute__((aligned(16))) uint8_t s_tab[GPB * 2 * kTabSlot];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wid = uniform(threadIdx.x >> 6);
  const uint32_t gi = wid / NT, w = wid % NT;          // group in the block, wave in the group
  const uint32_t nb = gridDim.x;                       // a multiple of 8 (launch_mac)
  uint32_t task = ((blockIdx.x & 7u) * (nb >> 3) + (blockIdx.x >> 3)) * GPB + gi;
  task = uniform(task);
  uint32_t cc, grp;
  const uint32_t ngrp = (a.nrowchunks + NT - 1) / NT;
  if (a.tile_fast) {
    grp = task % ngrp;
    task /= ngrp;
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
  } else {
    cc = task % a.ncolchunks;
    task /= a.ncolchunks;
    grp = task % ngrp;
    task /= ngrp;
  }
  uint32_t ks = 0;
  if (!DEC && a.ksplit > 1) {
    ks = task % a.ksplit;
    task /= a.ksplit;
  }
  const uint32_t g = task;
  // a group with nothing to do still takes part in the block's barriers (the other group's
  // steps): it runs k steps with no rows and builds nothing -- see bs_group's `idle`
  const uint32_t total = g < a.G ? (DEC ? const_load_u16(a.rows_per_gen + g) : a.rows) : 0u;
  const bool idle = grp * NT * 16u >= total;           // uniform over the group
  const uint32_t tile = grp * NT + w;
  const uint32_t row0 = tile * 16u;
  const uint32_t nrows = row0 < total ? min(16u, total - row0) : 0u;
  const uint32_t ring = lds_addr(s_raw + (gi * NT + w) * (kGrpRaw * kBsSlot));
  const uint32_t tabs = lds_addr(s_tab + gi * 2 * kTabSlot);
  const uint32_t i0 = ks * a.kpart;
  const uint32_t cnt = a.ksplit > 1 ? min(a.kpart, a.k - i0) : a.k;
  // every group of the block runs the same number of steps (a split-k part of another group may
  // be shorter: the block runs the longest part, shorter groups idle through the tail steps)
  const uint32_t steps = a.ksplit > 1 ? a.kpart : a.k;
  bs_group<NT, DEC, FULL>(a, idle ? 0u : g, tile, idle ? 0u : nrows, cc, lane, w, ring, tabs, i0, cnt,
                          steps, idle, ks ? a.kout + (ks - 1) * a.kout_step : a.out);
}

// Input row address of every plan position for the bit-sliced decode MAC: position i < k reads
// received source slot plan_in[i] (< k) or repair plan_in[i] - k; entries k .. k + kBsRing - 1
// repeat position k - 1 (the MAC's ring prefetches run past the last source).  Generations with
// nothing to decode are skipped (the MAC does not read them).
__global__ __launch_bounds__(256) void plan_rows(const uint16_t* __restrict__ plan_m,
                                                 const uint16_t* __restrict__ plan_in, uint32_t G,
                                                 uint32_t k, uint32_t r, uint64_t stride,
                                                 const uint8_t* src, const uint8_t* rep,
                                                 uint64_t* __restrict__ rows)
{
  const uint32_t kp = k + kBsRing;
  const uint64_t idx = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  if (idx >= static_cast<uint64_t>(G) * kp) return;
  const uint32_t g = static_cast<uint32_t>(idx / kp), i = static_cast<uint32_t>(idx % kp);
  if (plan_m[g] == 0) return;
  const uint32_t ii = plan_in[static_cast<size_t>(g) * k + (i < k ? i : k - 1)];
  const uint8_t* row = ii < k ? src + (static_cast<uint64_t>(g) * k + ii) * stride
                              : rep + (static_cast<uint64_t>(g) * r + (ii - k)) * stride;
  rows[idx] = reinterpret_cast<uint64_t>(row);
}

// Encode (DEC = false): rep[g][rows] = C_g * src[g]; decode (DEC = true): the plan's D_g applied to
// [repairs ; received sources], written into the lost source slots.  Each wave picks the
// smallest row tile covering its rows (wave-uniform branch), so no per-row guards in the loop.
template <int D, bool DEC>
__global__ __launch_bounds__(256) void gf_mac(MacArgs a)
{
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t task = uniform(blockIdx.x * kWaves + (threadIdx.x >> 6));
  const uint32_t cc = task % a.ncolchunks;
  task /= a.ncolchunks;
  const uint32_t rc = task % a.nrowchunks;
  const uint32_t g = task / a.nrowchunks;
  if (g >= a.G) return;
  const uint32_t total = DEC ? const_load_u16(a.rows_per_gen + g) : a.rows;
  const uint32_t row0 = rc * 32u;
  if (row0 >= total) return;
  const uint32_t nrows = min(32u, total - row0);
  const uint32_t col = cc * (256u * D) + lane * (4u * D);
  const bool active = col < a.stride;
  if (nrows > 16) mac_tile<32, D, DEC>(a, g, row0, nrows, col, active);
  else if (nrows > 8) mac_tile<16, D, DEC>(a, g, row0, nrows, col, active);
  else if (nrows > 4) mac_tile<8, D, DEC>(a, g, row0, nrows, col, active);
  else mac_tile<4, D, DEC>(a, g, row0, nrows, col, active);
}

// Encode preparation, one block per generation: the reference coefficient matrix
// (galois_field.hh:143-158, uint32 wraparound) as [k][rp] bytes, the encoded sizes
// (detail/encoder.cc:38, 61-62: XOR of bytewise-coded u16 lengths) and the repair symbol length
// (max source length, detail/encoder.cc:26, 44-48).
// c * x for the four bytes of x with a per-lane coefficient table (v_perm 3/3/2 split).
__device__ __forceinline__ uint32_t mul4(const uint32_t* t, uint32_t x)
{
  return bxor3(__builtin_amdgcn_perm(t[1], t[0], x & 0x07070707u),
               __builtin_amdgcn_perm(t[3], t[2], (x >> 3) & 0x07070707u),
               __builtin_amdgcn_perm(t[4], t[4], (x >> 6) & 0x03030303u));
}

struct PrepArgs {
  uint32_t G, k, r, rp;
  const uint16_t* src_len;
  const uint32_t* sid_base;
  const uint32_t* rid_base;
  uint8_t* coef;
  uint16_t* rep_size;
  uint16_t* rep_len;
  uint8_t* pair;               // non-null: try to pair generation g with g + kPairGap
};

// Generation pairing for the encode MAC (symbols of at most half a bit-sliced span): with
// continuous ids (sid = g*k + i, rid = g*r + j) the coefficient of generation g + 255 is that of g
// unless the uint32 product wraps a different number of times (galois_field.hh:143-158; 2^32 = 1
// mod 255), so most generations g with (g / 255) even share their matrix with g + 255.  encode_prep
// compares the two matrices; equal ones are encoded by one MAC wave, g's symbols in the first
// half of each lane's span and the partner's in the second.
constexpr uint32_t kPairGap = 255;

// Coefficients of one repair row along sources i, i + step, ... without multiplies:
// P = (R1 + S1) * R1 mod 2^32 grows by D = step * R1 per step, and since 2^32 = 1 (mod 255) the
// residue p = P mod 255 follows as p + (D mod 255) - carry(P + D).  coefficient = p + 1
// (galois_field.hh:143-158).
struct CoefWalk {
  uint32_t P, p, D, d;
  __device__ __forceinline__ CoefWalk(uint32_t R1, uint32_t S1, uint32_t step)
      : P((R1 + S1) * R1), D(step * R1)
  {
    p = P % 255u;
    d = D % 255u;
  }
  __device__ __forceinline__ uint32_t coef() const { return p + 1u; }
  __device__ __forceinline__ void next()
  {
    const uint32_t nP = P + D;
    const uint32_t t = p + d + (nP < P ? 254u : 255u);   // in [254, 763]
    const uint32_t t1 = min(t, t - 255u);
    p = min(t1, t1 - 255u);
    P = nP;
  }
};

// One wave per generation, four generations per 256-thread block (one LDS table copy for the
// four).  Lane = (coefficient word w of a source row = rows 4w..4w+3, source slot q): the lane
// walks sources q, q + nq, ..., writes its coefficient words and XORs the coded lengths of its
// sources into the four rows' encoded sizes; the slots' partial sizes are reduced through the
// wave's LDS slice.  No block-wide barrier after the table copy.
__global__ __launch_bounds__(256) void encode_prep(PrepArgs a)
{
  // LDS copy of the v_perm tables (encoded sizes), made only when some generation of the block
  // has unequal source lengths (one product per source and row) and k * r >= 1024; otherwise
  // the few lookups read the constant bank.
  __shared__ __attribute__((aligned(16))) uint32_t ptab[256][8];
  __shared__ uint16_t part[4][256];
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t g = blockIdx.x * 4u + wv;
  const bool live = g < a.G;
  const uint16_t* len = a.src_len + static_cast<size_t>(live ? g : 0u) * a.k;
  // id bases (and the pairing partner's) first: their loads overlap the length pass
  const uint32_t sidb = a.sid_base ? a.sid_base[live ? g : 0u] : g * a.k;
  const uint32_t ridb = a.rid_base ? a.rid_base[live ? g : 0u] : g * a.r;
  // pairing: a first-of-pair generation also walks its partner's coefficients and compares them
  // (only when the partner's id bases are congruent mod 255, the necessary condition)
  const bool first = live && a.pair && (g / kPairGap) % 2u == 0u;
  const bool has_partner = first && g + kPairGap < a.G;
  uint32_t psidb = 0, pridb = 0;
  if (has_partner) {
    const uint32_t gp = g + kPairGap;
    psidb = a.sid_base ? a.sid_base[gp] : gp * a.k;
    pridb = a.rid_base ? a.rid_base[gp] : gp * a.r;
  }
  // source lengths: max (the repair length) and whether they are all equal -- then a repair's
  // encoded size is multiply_size(L, XOR of its coefficients) (the product distributes over XOR),
  // one product per repair instead of one per source
  uint32_t lmax = 0, lmin = 0xFFFFu;
  for (uint32_t i = lane; live && i < a.k; i += 64u) {
    const uint32_t l = len[i];
    lmax = max(lmax, l);
    lmin = min(lmin, l);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lmax = max(lmax, static_cast<uint32_t>(__shfl_xor(lmax, o)));
    lmin = min(lmin, static_cast<uint32_t>(__shfl_xor(lmin, o)));
  }
  const bool same_len = !live || uniform(lmin) == uniform(lmax);
  const bool lds_tabs = __syncthreads_or(!same_len) && a.k * a.r >= 1024u;
  if (lds_tabs) {                                 // uniform
    const uint4* src = reinterpret_cast<const uint4*>(&d_perm.w[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(&ptab[0][0]);
    for (uint32_t i = threadIdx.x; i < 512u; i += 256u) dst[i] = src[i];
    __syncthreads();
  }
  const uint32_t (*tabs)[8] = lds_tabs ? ptab : d_perm.w;
  if (!live) return;
  uint16_t* pw = part[wv];
  const bool cmp = has_partner && psidb % 255u == sidb % 255u && pridb % 255u == ridb % 255u;
  uint32_t diff = 0;
  // Rows go in chunks of at most 256 (64 coefficient words): one chunk whenever r <= 256.
  const uint32_t nwt = a.rp >> 2;                 // rp % 4 == 0
  for (uint32_t wb = 0; wb < nwt; wb += 64u) {
  const uint32_t nw = min(nwt - wb, 64u);
  const uint32_t nq = 64u / nw;                   // source slots
  const uint32_t w = wb + lane % nw, q = lane / nw;
  const uint32_t cr = 4u * nw;                    // this chunk's rows: [4 * wb, 4 * wb + cr)
  if (q < nq) {
    uint8_t* coef = a.coef + static_cast<size_t>(g) * a.k * a.rp + 4u * w;
    CoefWalk cw[4] = {CoefWalk(ridb + 4u * w + 1u, sidb + q + 1u, nq),
                      CoefWalk(ridb + 4u * w + 2u, sidb + q + 1u, nq),
                      CoefWalk(ridb + 4u * w + 3u, sidb + q + 1u, nq),
                      CoefWalk(ridb + 4u * w + 4u, sidb + q + 1u, nq)};
    CoefWalk cp[4] = {CoefWalk(pridb + 4u * w + 1u, psidb + q + 1u, nq), CoefWalk(pridb + 4u * w + 2u, psidb + q + 1u, nq),
                      CoefWalk(pridb + 4u * w + 3u, psidb + q + 1u, nq), CoefWalk(pridb + 4u * w + 4u, psidb + q + 1u, nq)};
    uint32_t esz[4] = {0, 0, 0, 0};
    uint32_t csum = 0;                            // same_len: XOR of the coefficient words
    // four sources per pass, their lengths loaded together (one memory round trip per 4)
    for (uint32_t ib = q; ib < a.k; ib += 4u * nq) {
      uint32_t lq[4] = {0, 0, 0, 0};
      if (!same_len) {
#pragma unroll
        for (uint32_t e = 0; e < 4; ++e) lq[e] = ib + e * nq < a.k ? len[ib + e * nq] : 0u;
      }
#pragma unroll
      for (uint32_t e = 0; e < 4; ++e) {
        const uint32_t i = ib + e * nq;
        if (i >= a.k) break;
        uint32_t word = 0, pword = 0;
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          if (4u * w + b < a.r) {                 // rows >= r stay zero
            const uint32_t c = cw[b].coef();
            word |= c << (8 * b);
            // both length bytes times c in one v_perm lookup (galois_field.hh:108-115 codes a
            // u16 as a 2-byte region; a zero length stays zero)
            if (!same_len) esz[b] ^= mul4(tabs[c], lq[e]);
            if (cmp) pword |= cp[b].coef() << (8 * b);
          }
          cw[b].next();
          if (cmp) cp[b].next();
        }
        csum ^= word;
        diff |= word ^ pword;
        *reinterpret_cast<uint32_t*>(coef + static_cast<size_t>(i) * a.rp) = word;
      }
    }
    if (same_len) {
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) esz[b] = mul4(tabs[(csum >> (8 * b)) & 0xFFu], lmax);
    }
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) pw[q * cr + 4u * (w - wb) + b] = static_cast<uint16_t>(esz[b]);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  // pw holds nq * cr <= 256 partial sizes
  for (uint32_t j = lane; j < cr && 4u * wb + j < a.r; j += 64u) {
    uint16_t e = 0;
    for (uint32_t s2 = 0; s2 < nq; ++s2) e ^= pw[s2 * cr + j];
    a.rep_size[static_cast<size_t>(g) * a.r + 4u * wb + j] = e;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();                // the next chunk reuses pw
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (first) {
    const bool same = cmp && __ballot(diff != 0) == 0;
    if (lane == 0) {
      a.pair[g] = same ? 1 : 0;
      if (has_partner) a.pair[g + kPairGap] = same ? 2 : 0;
    }
  }
  if (a.rep_len && lane == 0) a.rep_len[g] = static_cast<uint16_t>(lmax);   // max source length
}

// One 64-thread block (one wave) per generation.  Reproduces what ntc::detail::decoder does when
// a generation's received sources, then its received repairs, arrive in ascending id order:
//  * m == 0: every repair is useless (detail/decoder.cc:77-89);
//  * fewer received repairs than m: nothing decodes, repairs stay pending;
//  * m == 1: the first repair peels the source (:133-149 create_source_from_repair);
//  * m >= 2: the first m-1 repairs wait; each further repair triggers attempt_full_decoding
//    (:412-566) on {first m-1} + {it}; a singular matrix drops it (invert() always reports
//    index rows-1 = the newest repair, invert_matrix.cc:40-44; decoder.cc:448-468).
// The inverse is unique, so a Gauss-Jordan with any pivot order gives the reference's M^-1;
// singularity (rank) is pivot-order independent too.
struct PlanArgs {
  uint32_t G, k, r;
  uint16_t* src_len;
  const uint8_t* src_mask;
  const uint16_t* rep_size;
  const uint8_t* rep_mask;
  const uint32_t* sid_base;
  const uint32_t* rid_base;
  ntc_gf256_decode_status* status;
  uint16_t* plan_m;
  uint16_t* plan_in;
  uint16_t* plan_out;
  uint8_t* plan_coef;
  uint32_t rp;
  uint32_t big_rows, big_pitch;   // decode_plan_big: LDS matrix shape
  // decode_plan_w, when non-null: also write the decode MAC's input row addresses (what
  // plan_rows computes at apply time) for the buffers the apply will use
  uint64_t* rows_out;
  const uint8_t* rows_src;
  const uint8_t* rows_rep;
  uint64_t rows_stride;
  uint32_t m_cap;                 // decode_plan_big: > 0: defer generations with m > m_cap
  uint32_t deferred_only;         // decode_plan_big: only the generations an m_cap pass deferred
};

// D column of one received-source position j (one lane): D[s][j] = sum_q (M^-1)[s][q] * c(q, j)
// for the R (padded) output rows s.  The lane's coefficient c(q, j) selects its own v_perm table
// (one 32-byte row of d_perm per q); the wave-uniform bytes (M^-1)[s..s+3][q] are the data, so one
// mul4 yields four rows' products.  acc[w] = D[4w..4w+3][j], the byte order of the plan's
// position-major layout (pc[j][s]).
template <int R, int RM>
__device__ __forceinline__ void plan_dcol(uint32_t m, uint32_t j, uint32_t sidb,
                                          const uint32_t* rq1, const uint32_t (*minvT)[RM / 4],
                                          uint8_t* dst, uint32_t rp)
{
  const uint32_t S1 = sidb + j + 1u;
  uint32_t acc[R / 4];
#pragma unroll
  for (int w = 0; w < R / 4; ++w) acc[w] = 0;
#pragma unroll 4
  for (uint32_t q = 0; q < m; ++q) {
    const uint32_t R1 = rq1[q];
    const uint32_t c = ((R1 + S1) * R1) % 255u + 1u;   // galois_field.hh:143-158
    const uint4 ab = *reinterpret_cast<const uint4*>(&d_perm.w[c][0]);
    const uint32_t tf[5] = {ab.x, ab.y, ab.z, ab.w, d_perm.w[c][4]};
#pragma unroll
    for (int w = 0; w < R / 4; ++w) acc[w] ^= mul4(tf, minvT[q][w]);
  }
  uint32_t* d = reinterpret_cast<uint32_t*>(dst);      // rp is a multiple of 4
#pragma unroll
  for (int w = 0; w < R / 4; ++w)
    if (4u * w < rp) d[w] = acc[w];
  for (uint32_t t = R; t < rp; t += 4) d[t / 4] = 0;
  (void)m;
}

// RM = row bound of this instantiation (r <= RM): sizes LDS and registers to the launch, so
// small generations keep many waves per CU (the plan is latency-bound).
template <int RM>
__global__ __launch_bounds__(64) void decode_plan(PlanArgs a)
{
  constexpr int kPitchW = (2 * RM) / 4 + 1;   // dwords per augmented row (odd: no bank conflicts)
  constexpr int kChunk = 256;                 // received sources staged per pass
  __shared__ __attribute__((aligned(16))) uint8_t exp_t[512];
  __shared__ __attribute__((aligned(16))) uint8_t log_t[256];
  __shared__ uint32_t A[RM][kPitchW];          // augmented [M | I], row q = repair q
  __shared__ uint16_t miss[RM];
  __shared__ uint16_t recv[RM];
  __shared__ uint16_t reps[RM];
  __shared__ uint32_t minvT[RM][RM / 4];       // (M^-1)[s][q] bytes, [q][s]
  __shared__ uint32_t rq1[RM];
  __shared__ uint16_t rl[kChunk];
  __shared__ uint16_t sl[kChunk];
  __shared__ uint16_t rszL[RM];
  __shared__ uint32_t szs[RM];

  const uint32_t lane = threadIdx.x;
  const uint32_t g = blockIdx.x;
  {
    const uint4* fe = reinterpret_cast<const uint4*>(d_field.exp);
    const uint4* fl = reinterpret_cast<const uint4*>(d_field.log);
    const uint4 ve = lane < 32 ? fe[lane] : fl[(lane - 32) & 15];
    if (lane < 32) reinterpret_cast<uint4*>(exp_t)[lane] = ve;
    else if (lane < 48) reinterpret_cast<uint4*>(log_t)[lane - 32] = ve;
  }


  const uint32_t k = a.k, r = a.r;
  const uint32_t sidb = a.sid_base ? a.sid_base[g] : g * k;
  const uint32_t ridb = a.rid_base ? a.rid_base[g] : g * r;
  const uint8_t* smask = a.src_mask + static_cast<size_t>(g) * k;
  const uint8_t* rmask = a.rep_mask + static_cast<size_t>(g) * r;
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));
  uint32_t m = 0;
  for (uint32_t base = 0; base < k; base += 64) {
    const uint32_t idx = base + lane;
    const bool lost = idx < k && smask[idx] == 0;
    const uint64_t b = __ballot(lost);
    if (lost) {
      const uint32_t pos = m + __popcll(b & lt);
      if (pos < RM) miss[pos] = static_cast<uint16_t>(idx);
    }
    m += __popcll(b);
  }
  if (lane < r) rszL[lane] = a.rep_size[static_cast<size_t>(g) * r + lane];
  uint32_t nrecv = 0;
  for (uint32_t base = 0; base < r; base += 64) {
    const uint32_t idx = base + lane;
    const bool got = idx < r && rmask[idx] != 0;
    const uint64_t b = __ballot(got);
    if (got) {
      const uint32_t pos = nrecv + __popcll(b & lt);
      if (pos < RM) recv[pos] = static_cast<uint16_t>(idx);
    }
    nrecv += __popcll(b);
  }
  __syncthreads();

  ntc_gf256_decode_status st{};
  st.nb_missing = static_cast<uint16_t>(m);
  st.last_repair = 0xFFFF;
  uint32_t mm = 0;

  if (m == 0) {
    st.state = 1;
    st.nb_useless = static_cast<uint16_t>(nrecv);
  } else if (nrecv < m || m > static_cast<uint32_t>(RM)) {
    st.state = 2;
  } else {
    const uint32_t nw = (2 * m + 3) / 4;   // dwords per augmented row in use
    bool ok = false;
    uint32_t t = m - 1;
    for (; t < nrecv; ++t) {
      // Lane q builds row q: coefficients of the missing sources, then the identity block.
      if (lane < m) {
        const uint32_t rq = (lane + 1 < m) ? recv[lane] : recv[t];
        reps[lane] = static_cast<uint16_t>(rq);
        const uint32_t rid = ridb + rq;
        for (uint32_t w = 0; w < nw; ++w) {
          uint32_t word = 0;
          for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t c = 4 * w + b;
            uint32_t v = 0;
            if (c < m) v = coefficient(rid, sidb + miss[c]);
            else if (c < 2 * m) v = (c - m == lane) ? 1u : 0u;
            word |= v << (8 * b);
          }
          A[lane][w] = word;
        }
      }
      __syncthreads();
      bool singular = false;
      for (uint32_t p = 0; p < m; ++p) {
        const uint32_t pw = p >> 2, ps = 8 * (p & 3);
        const uint32_t f = (lane < m) ? (A[lane][pw] >> ps) & 0xFFu : 0u;
        const uint64_t b = __ballot(lane >= p && lane < m && f != 0);
        if (b == 0) { singular = true; break; }
        const uint32_t q = __ffsll(static_cast<unsigned long long>(b)) - 1;
        if (q != p) {
          for (uint32_t w = lane; w < nw; w += 64) {
            const uint32_t tmp = A[p][w];
            A[p][w] = A[q][w];
            A[q][w] = tmp;
          }
          __syncthreads();
        }
        // normalise row p by 1/pivot (uniform coefficient table)
        const uint32_t piv = (A[p][pw] >> ps) & 0xFFu;
        const uint32_t* ti = d_perm.w[exp_t[(255 - log_t[piv]) % 255]];
        for (uint32_t w = lane; w < nw; w += 64) A[p][w] = mul4(ti, A[p][w]);
        __syncthreads();
        // eliminate column p from every other row: lane = row, per-lane table of its factor
        const uint32_t fa = (lane < m && lane != p) ? (A[lane][pw] >> ps) & 0xFFu : 0u;
        if (fa != 0) {
          uint32_t tf[5];
#pragma unroll
          for (int e = 0; e < 5; ++e) tf[e] = d_perm.w[fa][e];
#pragma unroll 4
          for (uint32_t w = 0; w < nw; ++w) A[lane][w] ^= mul4(tf, A[p][w]);
        }
        __syncthreads();
      }
      if (!singular) { ok = true; break; }
      __syncthreads();
      if (t == m - 1 && t + 1 < nrecv) {
        // The first candidate failed.  Rather than a full Gauss-Jordan per further candidate
        // (decoder.cc:448-468 tries t = m, m+1, ... in turn), screen them all at once, as
        // decode_plan_big does: {first m-1 repairs} + {t} is invertible iff the first m-1 rows
        // are independent and row t lies outside their span.  Forward elimination of all
        // received rows over the m missing columns with pivots from rows 0..m-2 only leaves
        // each candidate reduced against that basis; the first nonzero one is the repair the
        // reference stops at (none: every candidate fails).
        const uint32_t nwl = (m + 3) / 4;
        if (lane < nrecv) {
          const uint32_t rid = ridb + recv[lane];
          for (uint32_t w = 0; w < nwl; ++w) {
            uint32_t word = 0;
            for (uint32_t b = 0; b < 4; ++b) {
              const uint32_t c = 4 * w + b;
              if (c < m) word |= coefficient(rid, sidb + miss[c]) << (8 * b);
            }
            A[lane][w] = word;
          }
        }
        __syncthreads();
        uint32_t rank = 0;
        for (uint32_t c = 0; c < m && rank + 1 < m; ++c) {
          const uint32_t cw = c >> 2, cs = 8 * (c & 3);
          const uint32_t f = lane < nrecv ? (A[lane][cw] >> cs) & 0xFFu : 0u;
          const uint64_t b = __ballot(lane >= rank && lane + 1 < m && f != 0);
          if (b == 0) continue;                       // no pivot in this column (uniform)
          const uint32_t q = __ffsll(static_cast<unsigned long long>(b)) - 1;
          if (q != rank) {
            for (uint32_t w = lane; w < nwl; w += 64) {
              const uint32_t tmp = A[rank][w];
              A[rank][w] = A[q][w];
              A[q][w] = tmp;
            }
            __syncthreads();
          }
          const uint32_t* ti = d_perm.w[field_inv_dev((A[rank][cw] >> cs) & 0xFFu)];
          for (uint32_t w = lane; w < nwl; w += 64) A[rank][w] = mul4(ti, A[rank][w]);
          __syncthreads();
          const uint32_t fa = (lane > rank && lane < nrecv) ? (A[lane][cw] >> cs) & 0xFFu : 0u;
          if (fa != 0) {
            uint32_t tf[5];
#pragma unroll
            for (int e = 0; e < 5; ++e) tf[e] = d_perm.w[fa][e];
            for (uint32_t w = 0; w < nwl; ++w) A[lane][w] ^= mul4(tf, A[rank][w]);
          }
          __syncthreads();
          ++rank;
        }
        uint32_t next = nrecv;                        // none: every candidate fails
        if (rank + 1 == m) {
          uint32_t nz = 0;
          if (lane + 1 >= m && lane < nrecv)
            for (uint32_t w = 0; w < nwl; ++w) nz |= A[lane][w];
          const uint64_t b = __ballot(nz != 0);
          if (b != 0) next = __ffsll(static_cast<unsigned long long>(b)) - 1;
        }
        __syncthreads();
        t = next - 1;                                 // the loop's ++t moves to `next`
      }
    }
    if (!ok) {
      st.state = 3;
      const uint32_t f = nrecv - m + 1;
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
    } else {
      st.state = 0;
      const uint32_t f = t - (m - 1);
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
      st.nb_decoded = static_cast<uint16_t>(m);
      st.nb_useless = static_cast<uint16_t>(nrecv - 1 - t);
      st.last_repair = recv[t];
      mm = m;
      uint16_t* pin = a.plan_in + static_cast<size_t>(g) * k;
      uint8_t* pc = a.plan_coef + static_cast<size_t>(g) * k * a.rp;
      uint16_t* pout = a.plan_out + static_cast<size_t>(g) * a.rp;
      const uint16_t* slen = a.src_len + static_cast<size_t>(g) * k;
      auto minv = [&](uint32_t s, uint32_t q) -> uint32_t {   // (M^-1)[s][q] = A[s][m + q]
        const uint32_t c = m + q;
        return (A[s][c >> 2] >> (8 * (c & 3))) & 0xFFu;
      };
      for (uint32_t s = lane; s < a.rp; s += 64) pout[s] = (s < m) ? miss[s] : 0;
      // Positions 0..m-1: the chosen repairs; D[s][q] = (M^-1)[s][q].  Lane = output row s.
      for (uint32_t q = 0; q < m; ++q) {
        if (lane == 0) pin[q] = static_cast<uint16_t>(k + reps[q]);
        if (lane < a.rp)
          pc[static_cast<size_t>(q) * a.rp + lane] = static_cast<uint8_t>(lane < m ? minv(lane, q) : 0u);
      }
      if (lane < m) {
        rq1[lane] = ridb + reps[lane] + 1u;
        szs[lane] = rszL[reps[lane]];           // becomes the reduced encoded size of repair q
      }
      const uint32_t R = m <= 8 ? 8u : m <= 16 ? 16u : m <= 32 ? 32u : 64u;   // <= RM
      for (uint32_t idx = lane; idx < m * (R / 4); idx += 64) {
        const uint32_t q = idx / (R / 4), s0 = 4 * (idx % (R / 4));
        uint32_t word = 0;
        for (uint32_t b = 0; b < 4; ++b)
          if (s0 + b < m) word |= minv(s0 + b, q) << (8 * b);
        minvT[q][s0 / 4] = word;
      }
      __syncthreads();
      // Positions m..k-1: received sources ascending; D[s][j] = sum_q (M^-1)[s][q] * c(rep_q, j),
      // computed as a small v_perm MAC (lane = 4 consecutive positions, x = their coefficients).
      uint32_t pos_base = m;
      for (uint32_t cbase = 0; cbase < k; cbase += kChunk) {
        const uint32_t cend = min(k, cbase + static_cast<uint32_t>(kChunk));
        uint32_t cnt = 0;
        for (uint32_t b2 = cbase; b2 < cend; b2 += 64) {
          const uint32_t j = b2 + lane;
          const bool got = j < cend && smask[j] != 0;
          const uint64_t bb = __ballot(got);
          if (got) {
            rl[cnt + __popcll(bb & lt)] = static_cast<uint16_t>(j);
            sl[cnt + __popcll(bb & lt)] = slen[j];
          }
          cnt += __popcll(bb);
        }
        __syncthreads();
        for (uint32_t t2 = lane; t2 < cnt; t2 += 64) pin[pos_base + t2] = rl[t2];
        // reduced encoded sizes (detail/decoder.cc:402-404): szs[q] ^= c(q, j) (x) len_j over the
        // chunk's received sources; lanes split the sources, a wave XOR-reduction per repair.
        // Lane q owns repair q; the two length bytes multiply independently (galois_field.hh:
        // 108-115), so one mul4 with the lane's table for c(q, j) codes a whole u16 length.
        if (lane < m) {
          const uint32_t R1 = rq1[lane];
          uint32_t e = 0;
#pragma unroll 4
          for (uint32_t t2 = 0; t2 < cnt; ++t2) {
            const uint32_t c = ((R1 + sidb + rl[t2] + 1u) * R1) % 255u + 1u;
            const uint4 ab = *reinterpret_cast<const uint4*>(&d_perm.w[c][0]);
            const uint32_t tf[5] = {ab.x, ab.y, ab.z, ab.w, d_perm.w[c][4]};
            e ^= mul4(tf, sl[t2]);
          }
          szs[lane] ^= e;
        }
        for (uint32_t p0 = lane; p0 < cnt; p0 += 64) {
          uint8_t* dst = pc + static_cast<size_t>(pos_base + p0) * a.rp;
          const uint32_t j = rl[p0];
          if (R == 8 || RM == 8) plan_dcol<8, RM>(m, j, sidb, rq1, minvT, dst, a.rp);
          else if constexpr (RM >= 16) {
            if (R == 16 || RM == 16) plan_dcol<16, RM>(m, j, sidb, rq1, minvT, dst, a.rp);
            else if constexpr (RM >= 32) {
              if (R == 32 || RM == 32) plan_dcol<32, RM>(m, j, sidb, rq1, minvT, dst, a.rp);
              else if constexpr (RM >= 64) plan_dcol<64, RM>(m, j, sidb, rq1, minvT, dst, a.rp);
            }
          }
        }
        pos_base += cnt;
        __syncthreads();
      }
      // decoded size of missing source s = sum_q (M^-1)[s][q] (x) reduced size of repair q
      uint32_t sz = 0;
      if (lane < m)
#pragma unroll 4
        for (uint32_t q = 0; q < m; ++q) {
          const uint32_t c = minv(lane, q);
          const uint4 ab = *reinterpret_cast<const uint4*>(&d_perm.w[c][0]);
          const uint32_t tf[5] = {ab.x, ab.y, ab.z, ab.w, d_perm.w[c][4]};
          sz ^= mul4(tf, szs[q]);
        }
      if (lane < m) a.src_len[static_cast<size_t>(g) * k + miss[lane]] = static_cast<uint16_t>(sz);
    }
  }
  if (lane == 0) {
    a.plan_m[g] = static_cast<uint16_t>(mm);
    a.status[g] = st;
  }
}

// ------------------------------------------------------------ decode plan, 64 < r <= 255 ----
// Large windows (m up to 255, the w = 8 limit): one 256-thread workgroup per
// generation, the augmented matrix [M | I] (m x 2m bytes) in LDS with thread = row.  Same
// greedy retry (decoder.cc:448-468), status, decoded sizes (:484-497) and plan layout as
// decode_plan (the decode MAC reads the plan through plan_rows' row addresses).
// Windows this large are rare, so this kernel favours simplicity over speed (block barriers per
// pivot), but every step stays on the device.
constexpr uint32_t kBigRows = 255;
// decode_plan_big sizes its LDS matrix for m <= kBigCap first (several workgroups per CU); the
// generations with more missing sources are marked with this state and planned by a second,
// full-size launch that skips every other generation
constexpr uint32_t kBigCap = 64;
constexpr uint8_t kPlanDeferred = 0x80;

__global__ __launch_bounds__(256) void decode_plan_big(PlanArgs a)
{
  extern __shared__ __attribute__((aligned(16))) uint32_t big_lds[];
  // A: a.big_rows rows (>= r) of a.big_pitch dwords (>= 2r bytes, odd: conflict-free per row),
  // sized per launch so small windows fit several workgroups per CU
  if (a.deferred_only && a.status[blockIdx.x].state != kPlanDeferred) return;   // uniform
  const uint32_t P = a.big_pitch;
  uint32_t* A = big_lds;
  uint16_t* miss = reinterpret_cast<uint16_t*>(big_lds + a.big_rows * P);  // [256]
  uint16_t* recv = miss + 256;                                             // [256]
  uint16_t* reps = recv + 256;                                             // [256]
  uint16_t* rl = reps + 256;                                               // [256] chunk list
  uint16_t* sl = rl + 256;                                                 // [256] its lengths
  uint16_t* pivrow = sl + 256;                                             // [256] row of pivot col
  uint32_t* szs = reinterpret_cast<uint32_t*>(pivrow + 256);               // [256]
  uint32_t* wcnt = szs + 256;                                              // [4] + [1] (+3)
  uint32_t* wmin = wcnt + 8;                                               // [2][4] pivot votes
  uint32_t (*ptab)[8] = reinterpret_cast<uint32_t (*)[8]>(wcnt + 16);      // v_perm tables, 8 KiB
  uint32_t* c4 = &ptab[0][0] + 256 * 8;       // [m][8]: c(q, j) of 32 received positions, packed
  {   // per-thread coefficients index the tables divergently: serve them from LDS
    const uint4* src = reinterpret_cast<const uint4*>(&d_perm.w[0][0]);
    uint4* dst = reinterpret_cast<uint4*>(&ptab[0][0]);
    for (uint32_t i = threadIdx.x; i < 512u; i += 256u) dst[i] = src[i];
  }

  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t g = blockIdx.x;
  const uint32_t k = a.k, r = a.r;
  const uint32_t sidb = a.sid_base ? a.sid_base[g] : g * k;
  const uint32_t ridb = a.rid_base ? a.rid_base[g] : g * r;
  const uint8_t* smask = a.src_mask + static_cast<size_t>(g) * k;
  const uint8_t* rmask = a.rep_mask + static_cast<size_t>(g) * r;
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

  // Ordered block-wide compaction of the indices in [base, base + 256) satisfying `pred`, appended
  // to out[] from position `n` (entries past `cap` are dropped); returns how many satisfied it.
  auto compact = [&](uint32_t base, uint32_t end, bool lost, const uint8_t* msk, uint16_t* out,
                     uint32_t n, uint32_t cap) -> uint32_t {
    const uint32_t idx = base + tid;
    const bool hit = idx < end && ((msk[idx] == 0) == lost);
    const uint64_t b = __ballot(hit);
    if (lane == 0) wcnt[wv] = __popcll(b);
    __syncthreads();
    uint32_t off = 0, tot = 0;
    for (uint32_t w = 0; w < 4; ++w) {
      if (w < wv) off += wcnt[w];
      tot += wcnt[w];
    }
    if (hit) {
      const uint32_t pos = n + off + __popcll(b & lt);
      if (pos < cap) out[pos] = static_cast<uint16_t>(idx);
    }
    __syncthreads();
    return tot;
  };

  uint32_t m = 0;
  for (uint32_t base = 0; base < k; base += 256) m += compact(base, k, true, smask, miss, m, 256);
  const uint32_t nrecv = compact(0, r, false, rmask, recv, 0, 256);

  ntc_gf256_decode_status st{};
  st.nb_missing = static_cast<uint16_t>(m);
  st.last_repair = 0xFFFF;
  uint32_t mm = 0;
  if (m == 0) {
    st.state = 1;
    st.nb_useless = static_cast<uint16_t>(nrecv);
  } else if (nrecv < m || m > kBigRows) {
    st.state = 2;
  } else if (a.m_cap && m > a.m_cap) {
    st.state = kPlanDeferred;                 // this launch's matrix rows are too short
  } else {
    const uint32_t nw = (2 * m + 3) / 4;
    auto byte_at = [&](uint32_t row, uint32_t c) -> uint32_t {
      return (A[(row) * P + (c >> 2)] >> (8 * (c & 3))) & 0xFFu;
    };
    // Lowest row index voted by the block: each wave posts its lowest `hit` lane to wmin[par][wv]
    // (double-buffered by `par`, so a wave racing ahead to the next vote cannot overwrite a slot
    // still being read), one barrier, every thread takes the minimum.  0xFFFFFFFF: no vote.
    auto vote = [&](bool hit, uint32_t par) -> uint32_t {
      const uint64_t b = __ballot(hit);
      if (lane == 0) wmin[par * 4 + wv] = b ? wv * 64u + (__ffsll(static_cast<long long>(b)) - 1) : 0xFFFFFFFFu;
      __syncthreads();
      return min(min(wmin[par * 4], wmin[par * 4 + 1]), min(wmin[par * 4 + 2], wmin[par * 4 + 3]));
    };
    // Gauss-Jordan on {first m-1 received repairs} + {received repair t} (decoder.cc:448-468
    // drops repair t when singular).  No row swaps and no per-pivot normalisation: the pivot of
    // column p is the lowest not-yet-pivot row with a nonzero there (pivrow[p]); every other row
    // subtracts (its entry / pivot) x the pivot row; two barriers per pivot.  At the end row
    // pivrow[s] is d * [e_s | (M^-1) row s]; each thread divides its own row by its d.
    auto attempt = [&](uint32_t t) -> bool {
      if (tid < m) {       // thread q builds row q: coefficients of the missing sources | identity
        const uint32_t rq = (tid + 1 < m) ? recv[tid] : recv[t];
        reps[tid] = static_cast<uint16_t>(rq);
        const uint32_t rid = ridb + rq;
        for (uint32_t w = 0; w < nw; ++w) {
          uint32_t word = 0;
          for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t c = 4 * w + b;
            uint32_t v = 0;
            if (c < m) v = coefficient(rid, sidb + miss[c]);
            else if (c < 2 * m) v = (c - m == tid) ? 1u : 0u;
            word |= v << (8 * b);
          }
          A[(tid) * P + (w)] = word;
        }
      }
      __syncthreads();
      bool used = false;
      uint32_t mycol = 0;
      for (uint32_t p = 0; p < m; ++p) {
        const uint32_t x = (tid < m) ? byte_at(tid, p) : 0u;
        const uint32_t q = vote(tid < m && !used && x != 0, p & 1u);
        if (q == 0xFFFFFFFFu) return false;           // uniform: singular
        if (tid == q) {
          used = true;
          mycol = p;
          pivrow[p] = static_cast<uint16_t>(q);
        } else if (x != 0) {
          const uint32_t fa = gmul(static_cast<uint8_t>(x), static_cast<uint8_t>(field_inv_dev(byte_at(q, p))));
          const uint32_t* tf0 = ptab[fa];
          const uint32_t tf[5] = {tf0[0], tf0[1], tf0[2], tf0[3], tf0[4]};
          for (uint32_t w = 0; w < nw; ++w) A[(tid) * P + (w)] ^= mul4(tf, A[(q) * P + (w)]);
        }
        __syncthreads();
      }
      if (tid < m) {                                  // normalise: own pivot entry -> 1
        const uint32_t* ti = d_perm.w[field_inv_dev(byte_at(tid, mycol))];
        const uint32_t tinv[5] = {ti[0], ti[1], ti[2], ti[3], ti[4]};
        for (uint32_t w = 0; w < nw; ++w) A[(tid) * P + (w)] = mul4(tinv, A[(tid) * P + (w)]);
      }
      __syncthreads();
      return true;
    };
    uint32_t t = m - 1;
    bool ok = attempt(t);
    if (!ok && t + 1 < nrecv) {
      // Screening (same outcome as trying t = m, m+1, ... with a full Gauss-Jordan each, as
      // decoder.cc:448-468 does): {first m-1 repairs} + {t} is invertible iff the first m-1 rows
      // are independent and row t is outside their span.  One forward elimination over all
      // received rows (pivots chosen among the first m-1 only) leaves every candidate row
      // reduced against that basis; the first nonzero one is the repair that completes
      // decoding (none: every candidate fails).
      __syncthreads();
      const uint32_t nwl = (m + 3) / 4;
      if (tid < nrecv) {   // row i: received repair i over the missing sources
        const uint32_t rid = ridb + recv[tid];
        for (uint32_t w = 0; w < nwl; ++w) {
          uint32_t word = 0;
          for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t c = 4 * w + b;
            if (c < m) word |= coefficient(rid, sidb + miss[c]) << (8 * b);
          }
          A[(tid) * P + (w)] = word;
        }
      }
      __syncthreads();
      uint32_t rank = 0, par = 0;
      bool used = false;
      for (uint32_t c = 0; c < m && rank + 1 < m; ++c) {
        const uint32_t x = (tid < nrecv && !used) ? byte_at(tid, c) : 0u;
        const uint32_t q = vote(tid + 1 < m && !used && x != 0, par);
        par ^= 1u;
        if (q == 0xFFFFFFFFu) continue;               // no pivot in this column (uniform)
        if (tid == q) {
          used = true;
        } else if (x != 0) {                          // rows still in play: basis + candidates
          const uint32_t fa = gmul(static_cast<uint8_t>(x), static_cast<uint8_t>(field_inv_dev(byte_at(q, c))));
          const uint32_t* tf0 = ptab[fa];
          const uint32_t tf[5] = {tf0[0], tf0[1], tf0[2], tf0[3], tf0[4]};
          for (uint32_t w = 0; w < nwl; ++w) A[(tid) * P + (w)] ^= mul4(tf, A[(q) * P + (w)]);
        }
        __syncthreads();
        ++rank;
      }
      uint32_t next = nrecv;
      if (rank + 1 == m) {
        uint32_t nz = 0;
        if (tid + 1 >= m && tid < nrecv)
          for (uint32_t w = 0; w < nwl; ++w) nz |= A[(tid) * P + (w)];
        const uint32_t v = vote(nz != 0, par);
        next = v != 0xFFFFFFFFu ? v : nrecv;
      }
      __syncthreads();
      if (next < nrecv) {
        t = next;
        ok = attempt(t);                              // invertible by construction
      }
    }
    if (!ok) {
      st.state = 3;
      const uint32_t f = nrecv - m + 1;
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
    } else {
      st.state = 0;
      const uint32_t f = t - (m - 1);
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
      st.nb_decoded = static_cast<uint16_t>(m);
      st.nb_useless = static_cast<uint16_t>(nrecv - 1 - t);
      st.last_repair = recv[t];
      mm = m;
      const uint32_t rp = a.rp;
      uint16_t* pin = a.plan_in + static_cast<size_t>(g) * k;
      uint8_t* pc = a.plan_coef + static_cast<size_t>(g) * k * rp;
      uint16_t* pout = a.plan_out + static_cast<size_t>(g) * rp;
      uint16_t* slen = a.src_len + static_cast<size_t>(g) * k;
      auto minv = [&](uint32_t s, uint32_t q) -> uint32_t { return byte_at(pivrow[s], m + q); };
      for (uint32_t s = tid; s < rp; s += 256) pout[s] = (s < m) ? miss[s] : 0;
      // positions 0 .. m-1: the chosen repairs, D[s][q] = (M^-1)[s][q]; thread = output row s
      for (uint32_t q = 0; q < m; ++q) {
        if (tid == 0) pin[q] = static_cast<uint16_t>(k + reps[q]);
        for (uint32_t s = tid; s < rp; s += 256)
          pc[static_cast<size_t>(q) * rp + s] = static_cast<uint8_t>(s < m ? minv(s, q) : 0u);
      }
      // reduced encoded sizes (decoder.cc:402-404), accumulated per chunk below: thread q owns
      // repair q; one mul4 codes both bytes of a u16 length (galois_field.hh:108-115)
      uint32_t red = tid < m ? a.rep_size[static_cast<size_t>(g) * r + reps[tid]] : 0u;
      const uint32_t rid_t = tid < m ? ridb + reps[tid] : 0u;
      // positions m .. k-1: received sources ascending, D[s][j] = sum_q (M^-1)[s][q] c(q, j)
      uint32_t pos = m;
      for (uint32_t base = 0; base < k; base += 256) {
        const uint32_t cnt = compact(base, k, false, smask, rl, 0, 256);
        for (uint32_t i = tid; i < cnt; i += 256) {
          pin[pos + i] = rl[i];
          sl[i] = slen[rl[i]];
        }
        __syncthreads();
        if (tid < m)
          for (uint32_t i = 0; i < cnt; ++i) red ^= mul4(ptab[coefficient(rid_t, sidb + rl[i])], sl[i]);
        // 32 positions at a time: thread s takes the table of (M^-1)[s][q] once per q and
        // multiplies four positions' coefficients c(q, j..j+3) per mul4
        for (uint32_t i0 = 0; i0 < cnt; i0 += 32) {
          const uint32_t n32 = min(32u, cnt - i0);
          __syncthreads();                      // the previous block's c4 reads are done
          for (uint32_t e = tid; e < m * 8u; e += 256) {
            const uint32_t q = e >> 3, w = e & 7u;
            const uint32_t rid = ridb + reps[q];
            uint32_t word = 0;
            for (uint32_t b = 0; b < 4; ++b) {
              const uint32_t i = i0 + 4 * w + b;
              if (i < cnt) word |= coefficient(rid, sidb + rl[i]) << (8 * b);
            }
            c4[e] = word;
          }
          __syncthreads();
          for (uint32_t s = tid; s < rp; s += 256) {
            uint32_t acc[8];
#pragma unroll
            for (int w = 0; w < 8; ++w) acc[w] = 0;
            if (s < m)
              for (uint32_t q = 0; q < m; ++q) {
                const uint32_t* tq = ptab[minv(s, q)];
                const uint32_t tt[5] = {tq[0], tq[1], tq[2], tq[3], tq[4]};
                const uint4 lo = *reinterpret_cast<const uint4*>(c4 + q * 8);
                const uint4 hi = *reinterpret_cast<const uint4*>(c4 + q * 8 + 4);
                acc[0] ^= mul4(tt, lo.x); acc[1] ^= mul4(tt, lo.y);
                acc[2] ^= mul4(tt, lo.z); acc[3] ^= mul4(tt, lo.w);
                acc[4] ^= mul4(tt, hi.x); acc[5] ^= mul4(tt, hi.y);
                acc[6] ^= mul4(tt, hi.z); acc[7] ^= mul4(tt, hi.w);
              }
#pragma unroll
            for (int i = 0; i < 32; ++i)
              if (static_cast<uint32_t>(i) < n32)
                pc[static_cast<size_t>(pos + i0 + i) * rp + s] =
                    static_cast<uint8_t>(acc[i >> 2] >> (8 * (i & 3)));
          }
        }
        pos += cnt;
        __syncthreads();
      }
      if (tid < m) szs[tid] = red & 0xFFFFu;
      __syncthreads();
      // decoded size of missing source s = sum_q (M^-1)[s][q] (x) reduced size of repair q
      if (tid < m) {
        uint32_t sz = 0;
        for (uint32_t q = 0; q < m; ++q) sz ^= mul4(ptab[minv(tid, q)], szs[q]);
        slen[miss[tid]] = static_cast<uint16_t>(sz);
      }
    }
  }
  if (tid == 0) {
    a.plan_m[g] = static_cast<uint16_t>(mm);
    a.status[g] = st;
  }
}
// dynamic LDS of decode_plan_big: matrix + miss/recv/reps/rl (u16) + szs + counters + v_perm tables
// (big_rows * big_pitch is padded to a multiple of 4 dwords, so ptab stays 16-byte aligned)
inline size_t big_lds_bytes(uint32_t rows, uint32_t pitch, uint32_t mmax)
{
  // A, miss/recv/reps/rl/sl/pivrow (6 x 256 u16), szs, wcnt + wmin, v_perm tables, c4 [mmax][8]
  return (static_cast<size_t>(rows) * pitch + 6 * 128 + 256 + 16 + 256 * 8 + mmax * 8) * 4;
}

// ------------------------------------------------------------- decode plan, r <= 32 (v2) ----
// Register-resident decode_plan for r <= 32 (config 3 and every shape with at most 32 repairs):
// one wave per generation, four generations per block sharing one LDS copy of the v_perm tables.
// Column layout: lane c < 2m holds column c of the augmented matrix [M | I] in W = RM/4 dwords
// (rows packed four per dword), so a Gauss-Jordan step is a rank-1 update of every lane's own
// registers: F = column p (v_readlane broadcast), y_c = A[p][c] / piv (one mul4 with the
// inverse's table), A[:, c] ^= F' * y_c with F'[p] = F[p] ^ 1, which leaves row p = y and clears
// column p elsewhere.  A zero on the diagonal (rare) swaps in the first nonzero row below it, as
// jerasure does (invert_matrix.cc:49-60); rank and M^-1 do not depend on the pivot order anyway.
// The decoded sizes use the same columns: dec_size[s] = sum_q Minv[s][q] (x) rsz_q ^ sum_j D[s][j]
// (x) len_j (decoder.cc:402-404, 484-497, linear in the bytes of each u16), each lane
// accumulating the terms of the columns it owns, then one XOR butterfly across the wave.
constexpr int kPlanWaves = 4;

__constant__ __attribute__((aligned(16))) PermTables d_pinv = make_inv_perm_tables();

// Byte i (runtime) of a register array.  Written as mask arithmetic, not as selects or an
// indexed access: LLVM turns the select-chain form back into a dynamically indexed array, which
// it can only keep in scratch memory.
template <int W>
__device__ __forceinline__ uint32_t byte_dyn(const uint32_t (&v)[W], uint32_t i)
{
  uint32_t x = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) x |= v[w] & (0u - static_cast<uint32_t>(static_cast<uint32_t>(w) == (i >> 2)));
  return (x >> (8u * (i & 3u))) & 0xFFu;
}

template <int W>
__device__ __forceinline__ void set_byte_dyn(uint32_t (&v)[W], uint32_t i, uint32_t b)
{
  const uint32_t sh = 8u * (i & 3u);
  const uint32_t bm = 0xFFu << sh, bv = (b & 0xFFu) << sh;
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const uint32_t sel = 0u - static_cast<uint32_t>(static_cast<uint32_t>(w) == (i >> 2));
    v[w] = (v[w] & ~(bm & sel)) | (bv & sel);
  }
}

// The same for a wave-uniform i: one indexed register move (s_set_gpr_idx) instead of a select
// per word, whose 64-bit lane masks were the plan's SGPR spills.
template <int W>
__device__ __forceinline__ uint32_t byte_dyn_u(const uint32_t (&v)[W], uint32_t i)
{
  return (v[i >> 2] >> (8u * (i & 3u))) & 0xFFu;
}

template <int W>
__device__ __forceinline__ void set_byte_dyn_u(uint32_t (&v)[W], uint32_t i, uint32_t b)
{
  const uint32_t sh = 8u * (i & 3u);
  v[i >> 2] = (v[i >> 2] & ~(0xFFu << sh)) | ((b & 0xFFu) << sh);
}

// The plan's v_perm tables in LDS, split by dword so that per-lane gathers spread over the banks:
// dwords 0-3 of c's table at a 16-byte pitch (ds_read_b128, 16 lanes per bank cycle: bank group c
// mod 16), dword 4 at a 4-byte pitch (ds_read_b32, 32 lanes: bank c mod 32).  With the 8-dword
// PermTables rows every b128 gather landed on c mod 8 and every fifth-dword gather on c mod 4.
// Rows 256 .. 259 repeat rows 1 .. 4: the table index of a coefficient straight from its folded
// residue (coef_tidx) reaches them for residues 255 .. 258.
struct PlanTab {
  uint4 a[260];
  uint32_t b[260];
};

// Table row of the coefficient ((R1 + S1) * R1 mod 2^32) mod 255 + 1 (galois_field.hh:143-158)
// without the divide: 256 = 1 (mod 255), so the byte sum of x is x mod 255 plus a multiple of 255;
// a second byte sum folds it to 0 .. 258, and rows 256 .. 259 of PlanTab repeat rows 1 .. 4.
__device__ __forceinline__ uint32_t coef_tidx(uint32_t R1, uint32_t S1)
{
  const uint32_t x = (R1 + S1) * R1;
  return __builtin_amdgcn_sad_u8(__builtin_amdgcn_sad_u8(x, 0u, 0u), 0u, 0u) + 1u;
}

// Gauss-Jordan step for column P (compile-time, so every register index is static): false when
// column P has no nonzero at or below row P (M singular).
template <int W, int P>
__device__ __forceinline__ bool gj_step(uint32_t (&col)[W], const PlanTab& ptab)
{
  constexpr uint32_t kNone = 0xFFFFFFFFu;
  constexpr int pw = P >> 2, ps = 8 * (P & 3);
  uint32_t F[W];
#pragma unroll
  for (int w = 0; w < W; ++w) F[w] = __builtin_amdgcn_readlane(col[w], P);
  uint32_t piv = (F[pw] >> ps) & 0xFFu;
  if (piv == 0) {
    // first row below P with a nonzero in column P (rows >= m are zero)
    uint32_t q = kNone;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t below = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if (4 * w + b > P) below |= 0x80u << (8 * b);
      const uint32_t f = F[w];
      const uint32_t nz = (((f & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | f) & below;
      if (q == kNone && nz != 0) q = 4u * w + (__builtin_ctz(nz) >> 3);
    }
    if (q == kNone) return false;
    const uint32_t bp = (col[pw] >> ps) & 0xFFu, bq = byte_dyn_u<W>(col, q);
    col[pw] = (col[pw] & ~(0xFFu << ps)) | (bq << ps);
    set_byte_dyn_u<W>(col, q, bp);
#pragma unroll
    for (int w = 0; w < W; ++w) F[w] = __builtin_amdgcn_readlane(col[w], P);
    piv = (F[pw] >> ps) & 0xFFu;
  }
  const uint32_t* ti = d_pinv.w[piv];
  const uint32_t tinv[5] = {ti[0], ti[1], ti[2], ti[3], ti[4]};
  const uint32_t y = mul4(tinv, (col[pw] >> ps) & 0xFFu);    // A[P][c] / piv
  const uint4 ab = ptab.a[y];
  const uint32_t ty[5] = {ab.x, ab.y, ab.z, ab.w, ptab.b[y]};
  F[pw] ^= 1u << ps;
#pragma unroll
  for (int w = 0; w < W; ++w)
    col[w] ^= mul4(ty, F[w]);
  return true;
}

template <int W, int P, int RM>
__device__ __forceinline__ bool gj_pivots(uint32_t (&col)[W], const PlanTab& ptab)
{
  if constexpr (P == RM) {
    return true;
  } else {
    if (!gj_step<W, P>(col, ptab)) return false;
    return gj_pivots<W, P + 1, RM>(col, ptab);
  }
}

#ifdef NTC_PLAN_CLOCK
__device__ uint64_t g_dbg_clk[1 << 18];
extern "C" int ntc_dbg_plan_clock(uint64_t* out, uint32_t n)
{
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg_clk), n * 8) == hipSuccess ? 0 : -1;
}
#define DBG_CLK(slot) uint64_t dbg_t##slot = wall_clock64()
#else
#define DBG_CLK(slot)
#endif

// A kernel-argument field loaded where it is used (the argument block starts the kernarg segment):
// the opaque offset keeps the compiler from hoisting every field to the kernel entry and holding
// them in SGPRs across the unrolled Gauss-Jordan steps, where they were spilled.
template <typename T>
__device__ __forceinline__ T late_arg(uint32_t off)
{
  asm volatile("" : "+s"(off));
  return const_load<T>(reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(__builtin_amdgcn_kernarg_segment_ptr())) + off);
}
#define NTC_PLAN_ARG(field) late_arg<decltype(PlanArgs::field)>(offsetof(PlanArgs, field))

template <int RM>
__global__ __launch_bounds__(64 * kPlanWaves) void decode_plan_w(PlanArgs a)
{
  DBG_CLK(0);
  static_assert(RM == 8 || RM == 16 || RM == 32, "the column layout needs 2 * RM <= 64 lanes");
  constexpr int W = RM / 4;
  __shared__ __attribute__((aligned(16))) PlanTab ptab;
  __shared__ uint16_t s_miss[kPlanWaves][RM];
  __shared__ uint16_t s_recv[kPlanWaves][RM];
  // scratch of the rank screening: received rows x (W + 1) dwords
  __shared__ __attribute__((aligned(16))) uint32_t s_scr[kPlanWaves][RM * (W + 1)];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wv = uniform(threadIdx.x >> 6);
  const uint32_t g0 = blockIdx.x * kPlanWaves + wv;
  const bool live = g0 < a.G;
  const uint32_t g = live ? g0 : 0u;      // a wave past G loads generation 0's words, then leaves
  const uint32_t k = a.k, r = a.r;
  const uint8_t* smask = a.src_mask + static_cast<size_t>(g) * k;
  const uint8_t* rmask = a.rep_mask + static_cast<size_t>(g) * r;
  // the first two 64-source chunks' masks and lengths, this generation's repair mask and sizes:
  // independent loads issued together, and together with the table fill below (one memory round
  // trip before the barrier instead of one per use; k <= 128 covers every generation of
  // configs 1-4)
  // (unconditional loads at clamped indices, selected at first use: a load under a lane branch
  // had its compare hoisted into the branch, which waited for the load right there)
  uint32_t smv[2], slv[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const uint32_t idx = 64u * c + lane, ci = min(idx, k - 1u);
    const uint32_t mv = smask[ci], lv = a.src_len[static_cast<size_t>(g) * k + ci];
    smv[c] = idx < k ? mv : 1u;
    slv[c] = idx < k ? lv : 0u;
  }
  // (r = 0: element 0 of the source arrays, a valid address, never used)
  const uint32_t ri = min(lane, max(r, 1u) - 1u);
  const uint8_t* rm = r ? rmask : smask;
  const uint16_t* rs = r ? a.rep_size + static_cast<size_t>(g) * r : a.src_len;
  const uint32_t rmv_l = rm[ri], rsv_l = rs[ri];
  const uint32_t rmv = lane < r ? rmv_l : 0u;
  const uint32_t rsv = lane < r ? rsv_l : 0u;
  const uint32_t sidb = a.sid_base ? a.sid_base[g] : g * k;
  const uint32_t ridb = a.rid_base ? a.rid_base[g] : g * r;
  for (uint32_t c = threadIdx.x; c < 260u; c += 64u * kPlanWaves) {
    const uint32_t e = c < 256u ? c : c - 255u;
    ptab.a[c] = *reinterpret_cast<const uint4*>(&d_perm.w[e][0]);
    ptab.b[c] = d_perm.w[e][4];
  }
  __syncthreads();   // the only block-wide barrier: the waves below are independent generations
  if (!live) return;
  uint16_t* miss = s_miss[wv];
  uint16_t* recv = s_recv[wv];
  uint32_t* scr = s_scr[wv];
  auto wave_sync = [] {    // LDS written by some lanes, read by others of the same wave
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto tab = [&](uint32_t c, uint32_t (&t)[5]) {
    const uint4 ab = ptab.a[c];
    uint32_t cb = c;                 // opaque: 4c by a shift, not 16c - 12c by a 64-bit mad
    asm volatile("" : "+v"(cb));
    t[0] = ab.x; t[1] = ab.y; t[2] = ab.z; t[3] = ab.w; t[4] = ptab.b[cb];
  };
  const uint64_t lt = (lane == 0) ? 0ull : ((~0ull) >> (64 - lane));

  auto mask_at = [&](uint32_t base) -> uint32_t {      // smask of source base + lane (or 1 past k)
    const uint32_t idx = base + lane;
    if (base == 0) return smv[0];
    if (base == 64) return smv[1];
    return idx < k ? smask[idx] : 1u;
  };
  uint32_t m = 0;
  for (uint32_t base = 0; base < k; base += 64) {
    const uint32_t idx = base + lane;
    const bool lost = idx < k && mask_at(base) == 0;
    const uint64_t b = __ballot(lost);
    if (lost) {
      const uint32_t pos = m + __popcll(b & lt);
      if (pos < RM) miss[pos] = static_cast<uint16_t>(idx);
    }
    m += __popcll(b);
  }
  uint32_t nrecv = 0;
  {
    const bool got = lane < r && rmv != 0;              // r <= RM <= 32
    const uint64_t b = __ballot(got);
    if (got) recv[__popcll(b & lt)] = static_cast<uint16_t>(lane);
    nrecv = __popcll(b);
  }
  wave_sync();

  ntc_gf256_decode_status st{};
  st.nb_missing = static_cast<uint16_t>(m);
  st.last_repair = 0xFFFF;
  uint32_t mm = 0;
  if (m == 0) {
    st.state = 1;
    st.nb_useless = static_cast<uint16_t>(nrecv);
  } else if (nrecv < m || m > static_cast<uint32_t>(RM)) {
    st.state = 2;
  } else {
    // lane q < nrecv: R1 of the q-th received repair; lane c < m: S1 of missing source c
    const uint32_t rid1 = lane < nrecv ? ridb + recv[lane] + 1u : 0u;
    const uint32_t S1 = lane < m ? sidb + miss[lane] + 1u : 0u;
    auto coef = [&](uint32_t R1) -> uint32_t {      // galois_field.hh:143-158
      return lane < m ? ((R1 + S1) * R1) % 255u + 1u : 0u;
    };
    // rows 0 .. m-2: the first m-1 received repairs; identity block in lanes m .. 2m-1
    uint32_t orig[W];
    // Columns (lanes) m .. RM-1 pad M to RM x RM with an identity block, so the Gauss-Jordan
    // always runs all RM pivots, with no per-m branch or per-word guard (block-diagonal: M^-1 is
    // unchanged, rows >= m stay zero in every other column); the augmented identity of the m
    // chosen repairs sits in lanes RM .. RM+m-1.  Lane indices come from opaque copies: compared
    // directly, their lane masks were shared with the emit phase's and stayed live across the
    // unrolled Gauss-Jordan as SGPR spills.
    uint32_t idl = lane - RM;
    asm volatile("" : "+v"(idl));
    uint32_t pdl = lane;
    asm volatile("" : "+v"(pdl));
    const uint32_t idr = idl < m ? idl : (pdl >= m && pdl < static_cast<uint32_t>(RM) ? pdl : ~0u);
    const uint32_t idb = idr != ~0u ? (1u << (8u * (idr & 3u))) : 0u, idw = idr >> 2;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const uint32_t q = 4u * w + b;
        if (q + 1 < m) v |= coef(__builtin_amdgcn_readlane(rid1, q)) << (8 * b);
      }
      orig[w] = v | (idw == static_cast<uint32_t>(w) ? idb : 0u);
    }
    // After a singular first candidate: rank screening instead of one Gauss-Jordan per further
    // candidate (decoder.cc:448-468 tries t = m, m+1, ... in turn).  {first m-1 repairs} + {t} is
    // invertible iff the first m-1 rows are independent and row t lies outside their span: a
    // forward elimination of all received rows over the m missing columns (lane = row, rows in
    // this wave's LDS scratch), pivots from rows 0..m-2 only,
    // leaves each candidate reduced against that basis; the first nonzero one is where the
    // reference stops.  Returns that candidate's index, or nrecv when every candidate fails.
    auto screen_candidates = [&]() -> uint32_t {
      constexpr uint32_t SP = W + 1;                   // odd dword pitch
      uint32_t* S = scr;
      const uint32_t nwl = (m + 3) / 4;
      if (lane < nrecv) {
        for (uint32_t w = 0; w < nwl; ++w) {
          uint32_t word = 0;
          for (uint32_t b = 0; b < 4; ++b) {
            const uint32_t c = 4 * w + b;
            if (c < m) {
              const uint32_t S1c = __builtin_amdgcn_readlane(S1, c);
              word |= (((rid1 + S1c) * rid1) % 255u + 1u) << (8 * b);
            }
          }
          S[lane * SP + w] = word;
        }
      }
      wave_sync();
      uint32_t rank = 0;
      for (uint32_t c = 0; c < m && rank + 1 < m; ++c) {
        const uint32_t cw = c >> 2, cs = 8 * (c & 3);
        const uint32_t f = lane < nrecv ? (S[lane * SP + cw] >> cs) & 0xFFu : 0u;
        const uint64_t b = __ballot(lane >= rank && lane + 1 < m && f != 0);
        if (b == 0) continue;                          // no pivot in this column (uniform)
        const uint32_t q = __ffsll(static_cast<unsigned long long>(b)) - 1;
        if (q != rank) {
          if (lane < nwl) {
            const uint32_t tmp = S[rank * SP + lane];
            S[rank * SP + lane] = S[q * SP + lane];
            S[q * SP + lane] = tmp;
          }
          wave_sync();
        }
        const uint32_t* ti = d_pinv.w[(S[rank * SP + cw] >> cs) & 0xFFu];
        const uint32_t tinv[5] = {ti[0], ti[1], ti[2], ti[3], ti[4]};
        if (lane < nwl) S[rank * SP + lane] = mul4(tinv, S[rank * SP + lane]);
        wave_sync();
        const uint32_t fa = (lane > rank && lane < nrecv) ? (S[lane * SP + cw] >> cs) & 0xFFu : 0u;
        if (fa != 0) {
          uint32_t tf[5];
          tab(fa, tf);
          for (uint32_t w = 0; w < nwl; ++w) S[lane * SP + w] ^= mul4(tf, S[rank * SP + w]);
        }
        wave_sync();
        ++rank;
      }
      uint32_t next = nrecv;
      if (rank + 1 == m) {
        uint32_t nz = 0;
        if (lane + 1 >= m && lane < nrecv)
          for (uint32_t w = 0; w < nwl; ++w) nz |= S[lane * SP + w];
        const uint64_t b = __ballot(nz != 0);
        if (b != 0) next = __ffsll(static_cast<unsigned long long>(b)) - 1;
      }
      wave_sync();
      return next;
    };
    uint32_t col[W];
    bool ok = false;
    uint32_t t = m - 1;
    DBG_CLK(1);
    // row m-1's byte of each word as a VGPR mask, made once: a uniform select per word here
    // became 64-bit lane masks that stayed live across the unrolled Gauss-Jordan (SGPR spills)
    const uint32_t shm = 8u * ((m - 1) & 3u);
    uint32_t selm[W];
#pragma unroll
    for (int w = 0; w < W; ++w) {
      uint32_t s_ = static_cast<uint32_t>(w) == ((m - 1) >> 2) ? ~0u : 0u;
      asm volatile("" : "+v"(s_));
      selm[w] = s_;
    }
    for (; t < nrecv; ++t) {
      // row m-1: received repair t (decoder.cc:448-468 retries with each newer repair); the
      // row holds only its identity bit in orig
      const uint32_t ct = coef(__builtin_amdgcn_readlane(rid1, t)) << shm;
#pragma unroll
      for (int w = 0; w < W; ++w) col[w] = orig[w] | (ct & selm[w]);
      if (gj_pivots<W, 0, RM>(col, ptab)) {
        ok = true;
        break;
      }
      if (t == m - 1 && t + 1 < nrecv) t = screen_candidates() - 1;   // the loop's ++t: next
    }
#ifdef NTC_PLAN_CLOCK
    uint64_t dbg_t2 = wall_clock64();
    if (lane == 0) { g_dbg_clk[8 * g + 1] = dbg_t1; g_dbg_clk[8 * g + 2] = dbg_t2; }
#endif
    if (!ok) {
      st.state = 3;
      const uint32_t f = nrecv - m + 1;
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
    } else {
      st.state = 0;
      const uint32_t f = t - (m - 1);
      st.nb_failed = static_cast<uint8_t>(f > 255 ? 255 : f);
      st.nb_decoded = static_cast<uint16_t>(m);
      st.nb_useless = static_cast<uint16_t>(nrecv - 1 - t);
      st.last_repair = recv[t];
      mm = m;
      const uint32_t rp = NTC_PLAN_ARG(rp);
      uint16_t* pin = NTC_PLAN_ARG(plan_in) + static_cast<size_t>(g) * k;
      uint8_t* pc = NTC_PLAN_ARG(plan_coef) + static_cast<size_t>(g) * k * rp;
      uint16_t* pout = NTC_PLAN_ARG(plan_out) + static_cast<size_t>(g) * rp;
      uint16_t* slen = NTC_PLAN_ARG(src_len) + static_cast<size_t>(g) * k;
      // plan row of input position `pos`: the rp coefficient bytes
      auto emit = [&](uint32_t pos, const uint32_t (&v)[W]) {
        uint32_t* d = reinterpret_cast<uint32_t*>(pc + static_cast<size_t>(pos) * rp);
#pragma unroll
        for (int w = 0; w < W; ++w)
          if (4u * w < rp) d[w] = v[w];
      };
      {   // every row word is computed: the words of rows >= m are zero (no per-word guards)
      uint32_t LO[W], HI[W];     // this lane's decoded-size terms, low and high length bytes
#pragma unroll
      for (int w = 0; w < W; ++w) LO[w] = HI[w] = 0;
      auto size_terms = [&](uint32_t len, const uint32_t (&v)[W]) {
        uint32_t tl[5], th[5];
        tab(len & 0xFFu, tl);
        tab(len >> 8, th);
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const uint32_t s0 = v[w] & 0x07070707u, s1 = (v[w] >> 3) & 0x07070707u;
            const uint32_t s2 = (v[w] >> 6) & 0x03030303u;
            LO[w] ^= xor3(__builtin_amdgcn_perm(tl[1], tl[0], s0), __builtin_amdgcn_perm(tl[3], tl[2], s1),
                          __builtin_amdgcn_perm(tl[4], tl[4], s2));
            HI[w] ^= xor3(__builtin_amdgcn_perm(th[1], th[0], s0), __builtin_amdgcn_perm(th[3], th[2], s1),
                          __builtin_amdgcn_perm(th[4], th[4], s2));
          }
      };
      // input row address of plan position `pos` (plan_rows' layout: k entries, then kBsRing
      // copies of the last one, read by the MAC's prefetch)
      uint64_t* const rows_o = NTC_PLAN_ARG(rows_out);
      uint64_t* rows_g = rows_o ? rows_o + static_cast<size_t>(g) * (k + kBsRing) : nullptr;
      auto put_row = [&](uint32_t pos, const uint8_t* row) {
        if (!rows_g) return;
        const uint64_t v = reinterpret_cast<uint64_t>(row);
        rows_g[pos] = v;
        if (pos == k - 1)
          for (uint32_t e = 0; e < static_cast<uint32_t>(kBsRing); ++e) rows_g[k + e] = v;
      };
      // R1 of the repair in row q (rows 0 .. m-2: received repairs 0 .. m-2; row m-1: repair t)
      const uint32_t t_rid1 = __builtin_amdgcn_readlane(rid1, t);
      const uint32_t row_r1 = (lane == m - 1) ? t_rid1 : rid1;
      // Positions 0 .. m-1: the chosen repairs, D[s][q] = Minv[s][q] = column m + q; the size of
      // each lane's repair from the preloaded sizes (shuffled with every lane active)
      const bool rep_lane = lane >= static_cast<uint32_t>(RM) && lane < RM + m;
      const uint32_t rq_l = rep_lane ? ((lane - RM + 1 < m) ? recv[lane - RM] : recv[t]) : 0u;
      const uint32_t rsz_l = __shfl(rsv, rq_l);
      if (rep_lane) {
        const uint32_t q = lane - RM;
        const uint32_t rq = rq_l;
        pin[q] = static_cast<uint16_t>(k + rq);
        put_row(q, NTC_PLAN_ARG(rows_rep) + (static_cast<uint64_t>(g) * r + rq) * NTC_PLAN_ARG(rows_stride));
        emit(q, col);
        size_terms(rsz_l, col);
      }
      if (lane < rp) pout[lane] = lane < m ? miss[lane] : 0;
      wave_sync();
      // Positions m .. k-1: received sources ascending, D[s][j] = sum_q Minv[s][q] * c(q, j).
      // Two 64-source chunks per pass (lane = source base + lane and base + 64 + lane): column
      // q's selector words are read across lanes and formed on the scalar unit once for both.
      // (k <= 64: one chunk, the pass without the second one's registers)
      uint32_t pos_base = m;
      auto emit_pass = [&](auto two_chunks) {
      constexpr bool kTwo = decltype(two_chunks)::value;
      for (uint32_t base = 0; base < k; base += 128) {
        const uint32_t j0 = base + lane, j1 = base + 64u + lane;
        const bool got0 = j0 < k && mask_at(base) != 0;
        const bool got1 = j1 < k && mask_at(base + 64u) != 0;
        const uint32_t len0 = base == 0 ? slv[0] : (got0 ? slen[j0] : 0u);
        const uint32_t len1 = base == 0 ? slv[1] : (got1 ? slen[j1] : 0u);
        const uint64_t b0 = __ballot(got0), b1 = __ballot(got1);
        const uint32_t pos0 = pos_base + __popcll(b0 & lt);
        const uint32_t pos1 = pos_base + __popcll(b0) + __popcll(b1 & lt);
        if (got0) {
          pin[pos0] = static_cast<uint16_t>(j0);
          put_row(pos0, NTC_PLAN_ARG(rows_src) + (static_cast<uint64_t>(g) * k + j0) * NTC_PLAN_ARG(rows_stride));
        }
        if (got1) {
          pin[pos1] = static_cast<uint16_t>(j1);
          put_row(pos1, NTC_PLAN_ARG(rows_src) + (static_cast<uint64_t>(g) * k + j1) * NTC_PLAN_ARG(rows_stride));
        }
        const bool two = kTwo && b1 != 0;                  // wave-uniform
        const uint32_t Sa = sidb + j0 + 1u, Sb = sidb + j1 + 1u;
        uint32_t acc0[W], acc1[W];
#pragma unroll
        for (int w = 0; w < W; ++w) acc0[w] = acc1[w] = 0;
        const uint32_t mq = m;
        // Column q's selector words, uniform: M^-1 column q is lane RM + q's col[] (read across
        // lanes), its v_perm selectors formed on the scalar unit.  Broadcast LDS reads of them
        // (6 x 16 B per lane and q) saturated the CU's LDS with 16 waves in this loop.
        auto selectors = [&](uint32_t q, uint32_t (&sq)[3][W]) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const uint32_t cw = __builtin_amdgcn_readlane(col[w], RM + q);
            sq[0][w] = cw & 0x07070707u;
            sq[1][w] = (cw >> 3) & 0x07070707u;
            sq[2][w] = (cw >> 6) & 0x03030303u;
          }
        };
        // Products of an even q and the next odd one share their XORs: the even step folds two of
        // its three lookups into acc and leaves the third pending, the odd step folds that one and
        // its own three (three bitop3 per word for two q instead of four).
        auto mac_even = [&](const uint32_t (&t)[5], const uint32_t (&sq)[3][W], uint32_t (&acc)[W],
                            uint32_t (&pend)[W]) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            acc[w] = xor3(acc[w], __builtin_amdgcn_perm(t[1], t[0], sq[0][w]),
                          __builtin_amdgcn_perm(t[3], t[2], sq[1][w]));
            pend[w] = __builtin_amdgcn_perm(t[4], t[4], sq[2][w]);
          }
        };
        auto mac_odd = [&](const uint32_t (&t)[5], const uint32_t (&sq)[3][W], uint32_t (&acc)[W],
                           const uint32_t (&pend)[W]) {
#pragma unroll
          for (int w = 0; w < W; ++w) {
            const uint32_t a = xor3(acc[w], pend[w], __builtin_amdgcn_perm(t[1], t[0], sq[0][w]));
            acc[w] = xor3(a, __builtin_amdgcn_perm(t[3], t[2], sq[1][w]),
                          __builtin_amdgcn_perm(t[4], t[4], sq[2][w]));
          }
        };
        // the coefficient tables of q + 1 are looked up while q's products are formed (their LDS
        // gathers are issued after q's selector reads, so their wait leaves them in flight); two
        // table sets alternate, so nothing is copied between iterations.  One loop per chunk
        // count (wave-uniform), so the second chunk's registers are not carried through phis.
        auto q_loop = [&](auto two_c) {
          constexpr bool kT = decltype(two_c)::value;
          auto tables = [&](uint32_t q, uint32_t (&t0)[5], uint32_t (&t1)[5]) {
            const uint32_t R1 = __builtin_amdgcn_readlane(row_r1, q);
            tab(coef_tidx(R1, Sa), t0);
            if constexpr (kT) tab(coef_tidx(R1, Sb), t1);
          };
          uint32_t tA0[5], tA1[5], tB0[5], tB1[5];
          uint32_t pend0[W], pend1[W];
          tables(0, tA0, tA1);
          for (uint32_t q = 0; q < mq; q += 2) {
            uint32_t sq[3][W];
            selectors(q, sq);
            if (q + 1 < mq) tables(q + 1, tB0, tB1);
            mac_even(tA0, sq, acc0, pend0);
            if constexpr (kT) mac_even(tA1, sq, acc1, pend1);
            if (q + 1 >= mq) {                     // odd m: the last pending lookups
#pragma unroll
              for (int w = 0; w < W; ++w) {
                acc0[w] ^= pend0[w];
                if constexpr (kT) acc1[w] ^= pend1[w];
              }
              break;
            }
            selectors(q + 1, sq);
            if (q + 2 < mq) tables(q + 2, tA0, tA1);
            mac_odd(tB0, sq, acc0, pend0);
            if constexpr (kT) mac_odd(tB1, sq, acc1, pend1);
          }
        };
        if (mq) {
          if (two) q_loop(std::true_type{});
          else q_loop(std::false_type{});
        }
        if (got0) {
          emit(pos0, acc0);
          size_terms(len0, acc0);
        }
        if (got1) {
          emit(pos1, acc1);
          size_terms(len1, acc1);
        }
        pos_base += __popcll(b0) + __popcll(b1);
      }
      };
      if (k > 64) emit_pass(std::true_type{});
      else emit_pass(std::false_type{});
      // XOR-reduce the size terms over the wave; lane s < m keeps byte s
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int w = 0; w < W; ++w) {
            LO[w] ^= __shfl_xor(LO[w], off);
            HI[w] ^= __shfl_xor(HI[w], off);
          }
      if (lane < m) {
        const uint32_t lo = byte_dyn<W>(LO, lane), hi = byte_dyn<W>(HI, lane);
        slen[miss[lane]] = static_cast<uint16_t>(lo | (hi << 8));
      }
      }
    }
  }
  if (lane == 0) {
    NTC_PLAN_ARG(plan_m)[g] = static_cast<uint16_t>(mm);
    NTC_PLAN_ARG(status)[g] = st;
#ifdef NTC_PLAN_CLOCK
    g_dbg_clk[8 * g + 0] = dbg_t0;
    g_dbg_clk[8 * g + 3] = wall_clock64();
    g_dbg_clk[8 * g + 4] = st.state;
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    g_dbg_clk[8 * g + 5] = hw;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    g_dbg_clk[8 * g + 6] = xcc;
#endif
  }
}

// ----------------------------------------------------------------------- region multiply ----
// ntc_gf256_gather_combine: one wave per (job, 1 KiB of its output); a lane owns 16 bytes.  The
// terms of a job are wave-uniform: their descriptors and the v_perm tables of their coefficients
// come through the scalar cache.
__global__ __launch_bounds__(64) void gather_combine(const ntc_gf256_gather_job* __restrict__ jobs,
                                                     const ntc_gf256_gather_term* __restrict__ terms)
{
  static_assert(sizeof(ntc_gf256_gather_job) == 32 && sizeof(ntc_gf256_gather_term) == 16, "layout");
  const u32x8 j8 = const_load<u32x8>(jobs + blockIdx.x);   // out (2 dwords), out2 (2), term0, nterms, len
  const u32x4 j4 = {j8[0], j8[1], j8[4], j8[5]};
  const uint32_t jlen = j8[6];
  uint8_t* out = reinterpret_cast<uint8_t*>((static_cast<uint64_t>(j4[1]) << 32) | j4[0]);
  uint8_t* out2 = reinterpret_cast<uint8_t*>((static_cast<uint64_t>(j8[3]) << 32) | j8[2]);
  const uint32_t col = blockIdx.y * 1024u + threadIdx.x * 16u;
  if (col >= ((jlen + 15u) & ~15u)) return;
  uint32_t acc[4] = {0, 0, 0, 0};
  // one term: its piece (zero past the term's length), times its coefficient, into acc
  auto piece = [&](const u32x4 t4) -> uint4 {
    const uint32_t tlen = t4[2];
    const uint8_t* src = reinterpret_cast<const uint8_t*>((static_cast<uint64_t>(t4[1]) << 32) | t4[0]);
    return col < tlen ? *reinterpret_cast<const uint4*>(src + col) : make_uint4(0, 0, 0, 0);
  };
  auto table = [&](const u32x4 t4, uint32_t (&tf)[5]) {
    const uint32_t* tb = d_perm.w[t4[3] & 0xFFu];
    tf[0] = tb[0]; tf[1] = tb[1]; tf[2] = tb[2]; tf[3] = tb[3]; tf[4] = tb[4];
  };
  auto add = [&](const u32x4 t4, const uint4 v, const uint32_t (&tf)[5]) {
    uint32_t x[4] = {v.x, v.y, v.z, v.w};
    const uint32_t tlen = t4[2];
    const uint32_t rem = tlen > col ? tlen - col : 0u;    // bytes of this piece that take part
    if (rem < 16u) {
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t keep = rem > 4u * d ? rem - 4u * d : 0u;
        x[d] &= keep >= 4u ? 0xFFFFFFFFu : (1u << (8u * keep)) - 1u;
      }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) acc[d] ^= mul4(tf, x[d]);
  };
  // four terms per step: their descriptors in one scalar load, then their four tables and four
  // pieces in flight together (a job's terms are a dependent chain of descriptor -> piece and
  // table loads otherwise)
  const uint32_t nt = j4[3], t0 = j4[2];
  uint32_t t = 0;
  for (; t + 4 <= nt; t += 4) {
    u32x4 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = const_load<u32x4>(terms + t0 + t + i);
    uint32_t tf[4][5];
#pragma unroll
    for (int i = 0; i < 4; ++i) table(d[i], tf[i]);
    uint4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = piece(d[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) add(d[i], v[i], tf[i]);
  }
  for (; t < nt; ++t) {
    const u32x4 d = const_load<u32x4>(terms + t0 + t);
    uint32_t tf[5];
    table(d, tf);
    add(d, piece(d), tf);
  }
  *reinterpret_cast<uint4*>(out + col) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
  if (out2) *reinterpret_cast<uint4*>(out2 + col) = make_uint4(acc[0], acc[1], acc[2], acc[3]);
}

__global__ __launch_bounds__(256) void region_mul(const uint8_t* __restrict__ src,
                                                  uint8_t* __restrict__ dst, size_t len,
                                                  uint32_t c, int add)
{
  const uint32_t* t = d_perm.w[c];
  const uint32_t a0 = t[0], a1 = t[1], b0 = t[2], b1 = t[3], e = t[4];
  const size_t nw = len / 4;
  const size_t gs = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t w = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; w < nw; w += gs) {
    uint32_t x;
    memcpy(&x, src + 4 * w, 4);
    const uint32_t p = xor3(__builtin_amdgcn_perm(a1, a0, x & 0x07070707u),
                            __builtin_amdgcn_perm(b1, b0, (x >> 3) & 0x07070707u),
                            __builtin_amdgcn_perm(e, e, (x >> 6) & 0x03030303u));
    uint32_t y = p;
    if (add) { uint32_t o; memcpy(&o, dst + 4 * w, 4); y ^= o; }
    memcpy(dst + 4 * w, &y, 4);
  }
  if (blockIdx.x == 0 && threadIdx.x < (len & 3)) {
    const size_t i = nw * 4 + threadIdx.x;
    const uint8_t v = gmul(static_cast<uint8_t>(c), src[i]);
    dst[i] = add ? static_cast<uint8_t>(dst[i] ^ v) : v;
  }
}

}  // namespace ntcgpu

// =================================================================================== C ABI ====
using namespace ntcgpu;

namespace ntcgpu {

thread_local std::string g_err;

int fail(int code, const std::string& msg)
{
  g_err = msg;
  return code;
}

int hip_check(hipError_t e, const char* what)
{
  if (e == hipSuccess) return NTC_GPU_OK;
  return fail(e == hipErrorOutOfMemory ? NTC_GPU_ENOMEM : NTC_GPU_EDEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace ntcgpu

namespace {

uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

// Column width per lane of the v_perm MAC.
int pick_d(uint32_t stride)
{
  // 8 B per lane measured fastest on MI355X for 1-4 KiB symbols (more waves per SIMD at the same
  // per-coefficient table cost); 4 B only when the stride forces it.
  return stride % 8 == 0 ? 2 : 1;
}

typedef void (*mac_fn)(MacArgs);

mac_fn pick_kernel(bool dec, int D)
{
  if (dec) return D == 4 ? gf_mac<4, true> : D == 2 ? gf_mac<2, true> : gf_mac<1, true>;
  return D == 4 ? gf_mac<4, false> : D == 2 ? gf_mac<2, false> : gf_mac<1, false>;
}

// MAC formulation for a stride.  The bit-sliced kernel spans 2 KiB per wave (two 16-byte pieces per
// lane), so short symbols leave lanes idle; measured on MI355X it beats the v_perm
// kernel (8-byte lanes) once >= ~1/3 of its lanes carry data (k=32 r=8, G=8192: 512 B symbols
// 606 vs 794 GiB/s, 768 B 888 vs 765, 1 KiB 1139 vs 999 -- bit-sliced vs v_perm).
// ntc_gf256_set_mac_kind forces one (results are identical).
bool use_bitslice(const ntc_gf256_engine* e, uint32_t stride)
{
  if (stride % 16 != 0) return false;
  if (e->mac_kind != NTC_GF256_MAC_AUTO)
    return e->mac_kind == NTC_GF256_MAC_BITSLICE || e->mac_kind == NTC_GF256_MAC_BITSLICE_GROUPED ||
           e->mac_kind == NTC_GF256_MAC_BITSLICE_PAIRED;
  const uint32_t pieces = stride / 16, spans = (stride + 2047) / 2048;   // 16-B pieces per span: 128
  return pieces * 100 >= spans * 128 * 33;
}

// Bit-sliced MAC kernel for a tile height and span shape (pair: the encode pairing form).
mac_fn pick_bs(bool dec, uint32_t rowtile, bool full, bool pair)
{
  if (pair) return rowtile == 16 ? gf_mac_bs<16, false, false, true> : gf_mac_bs<8, false, false, true>;
  if (rowtile == 16)
    return dec ? (full ? gf_mac_bs<16, true, true> : gf_mac_bs<16, true, false>)
               : (full ? gf_mac_bs<16, false, true> : gf_mac_bs<16, false, false>);
  return dec ? (full ? gf_mac_bs<8, true, true> : gf_mac_bs<8, true, false>)
             : (full ? gf_mac_bs<8, false, true> : gf_mac_bs<8, false, false>);
}

template <int J, int NS>
mac_fn pick_bsp_(bool dec, bool full)
{
  return dec ? (full ? gf_mac_bsp<J, NS, true, true> : gf_mac_bsp<J, NS, true, false>)
             : (full ? gf_mac_bsp<J, NS, false, true> : gf_mac_bsp<J, NS, false, false>);
}

mac_fn pick_bsp(bool dec, bool full, int j, int ns)
{
  if (j == 2) return ns == 4 ? pick_bsp_<2, 4>(dec, full) : pick_bsp_<2, 3>(dec, full);
  return ns == 4 ? pick_bsp_<1, 4>(dec, full) : pick_bsp_<1, 3>(dec, full);
}

mac_fn pick_bsg(bool dec, bool full)
{
  return dec ? (full ? gf_mac_bsg<2, true, true> : gf_mac_bsg<2, true, false>)
             : (full ? gf_mac_bsg<2, false, true> : gf_mac_bsg<2, false, false>);
}

// out ^= the split-k parts 1 .. nparts (16 B per thread and step, grid-stride)
__global__ __launch_bounds__(256) void ksplit_reduce(uint4* __restrict__ out, const uint4* __restrict__ parts,
                                                     uint64_t n16, uint32_t nparts)
{
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * 256u;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x; i < n16; i += step) {
    uint4 v = out[i];
    for (uint32_t p = 0; p < nparts; ++p) {
      const uint4 w = parts[p * n16 + i];
      v.x ^= w.x; v.y ^= w.y; v.z ^= w.z; v.w ^= w.w;
    }
    out[i] = v;
  }
}

// Bit-slice every 2 KiB span of a contiguous source block (stride % 2048 == 0) exactly as bs_tile's
// fill does in registers: lane l's pieces [16 l, +16) and [1024 + 16 l, +16) of a span become the
// 8 planes of transpose8, stored back in the same places, so gf_mac_bs<..., SL> loads planes
// where it loaded bytes.  One HBM pass (n bytes read, n written) in place of the 48-op transpose
// of every (source, 16-row tile) -- worth it once a source feeds many tiles (kSliceRows).
// n32 = bytes / 32: one (span, lane) item per thread and step, 1 KiB contiguous per wave access.
__global__ __launch_bounds__(256) void bs_preslice(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                   uint64_t n32)
{
  const uint64_t step = static_cast<uint64_t>(gridDim.x) * 256u;
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x; t < n32; t += step) {
    const uint64_t i0 = (t >> 6) * 128u + (t & 63u);
    const uint4 p = in[i0], q = in[i0 + 64];
    uint32_t y[8] = {p.x, p.y, p.z, p.w, q.x, q.y, q.z, q.w};
    transpose8(y);
    out[i0] = make_uint4(y[0], y[1], y[2], y[3]);
    out[i0 + 64] = make_uint4(y[4], y[5], y[6], y[7]);
  }
}

// Rows from which an encode / combine with whole spans pre-slices its sources.  Measured at
// config 5 (k = n = 1024, 64 KiB, profiles/r05/ab/preslice_config5.txt): the pass takes 0.025 ms
// for 64 MiB (0.76 ns per 2 KiB span) and each MAC drops 0.874 -> 0.776 ms over 64 row tiles
// (0.047 ns per span and 16-row tile), so it breaks even at ~16 tiles; 24 tiles keep a margin.
constexpr uint32_t kSliceRows = 384;

// Launch the region MAC over all (generation, row tile, column span) tasks of `a`.
int launch_mac(ntc_gf256_engine* e, bool dec, MacArgs& a, hipStream_t st, const char* what)
{
  mac_fn fn;
  uint32_t rowtile, span, wpb;
  uint64_t blk_align = 1;
  uint32_t group = 1;                           // 16-row tiles per workgroup sharing the fill
  bool paired = false;                          // gf_mac_bsp: tile pairs sharing the transpose
  if (a.pair || use_bitslice(e, a.stride)) {
    // 16-row tiles (3 waves per SIMD) once a tile has more than 8 rows to fill, else 8-row
    // tiles (4 waves per SIMD)
    rowtile = e->rowtile_force ? e->rowtile_force : a.rows > 8 ? 16u : 8u;
    span = 2048;
    wpb = kBsWaves;
    blk_align = 8;                              // the kernel's XCD renumbering
    fn = pick_bs(dec, rowtile, a.stride % 2048 == 0, a.pair != nullptr);
    if (!a.pair && rowtile == 16 && e->mac_kind == NTC_GF256_MAC_BITSLICE_GROUPED && a.rows > 16) {
      group = 2;                                // gf_mac_bsg: tile pairs share the source fill
      fn = pick_bsg(dec, a.stride % 2048 == 0);
    }
    if (!a.pair && rowtile == 16 && e->mac_kind == NTC_GF256_MAC_BITSLICE_PAIRED && a.rows > 16)
      paired = true;                            // gf_mac_bsp, unless sliced or split below
    // a tall encode / combine over whole spans: slice the sources once (bs_preslice) instead of
    // once per row tile
    if (!dec && !a.pair && group == 1 && a.stride % 2048 == 0 &&
        (e->slice_force >= 0 ? e->slice_force != 0 : a.rows >= kSliceRows)) {
      paired = false;
      const uint64_t n = static_cast<uint64_t>(a.G) * a.k * a.stride;
      // as for the split-k parts: a stream being captured must not allocate; and the copy is an
      // optimisation, so without room for it (hipMalloc fails) the MAC slices in registers
      hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
      const bool capturing = hipStreamIsCapturing(st, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
      if (n > e->slice_cap && !capturing) {
        void* p = nullptr;
        const size_t na = grow_to(e, n, e->slice_cap);
        if (hipMalloc(&p, na) == hipSuccess) {
          drop_buf(e, e->slice);
          e->slice = p;
          e->slice_cap = na;
        } else {
          (void)hipGetLastError();             // clear it: the call proceeds unsliced
        }
      }
      if (n <= e->slice_cap) {
        int rc;
        const uint64_t n32 = n / 32;
        const uint32_t nblk = static_cast<uint32_t>(std::min<uint64_t>((n32 + 255) / 256, 16384));
        {
          KernelTimer kt(e, NTC_GF256_K_SLICE, st, true);
          hipExtLaunchKernelGGL(bs_preslice, dim3(nblk), dim3(256), 0, st, kt.start(), kt.stop(), 0,
                                reinterpret_cast<const uint4*>(a.in0), static_cast<uint4*>(e->slice), n32);
        }
        if ((rc = hip_check(hipGetLastError(), "bs_preslice launch"))) return rc;
        a.in0 = static_cast<const uint8_t*>(e->slice);
        fn = rowtile == 16 ? gf_mac_bs<16, false, true, false, true> : gf_mac_bs<8, false, true, false, true>;
      }
    }
    if (dec && !a.row_ptr) {                   // (else the plan wrote the row addresses)
      const uint64_t nr = static_cast<uint64_t>(a.G) * (a.k + kBsRing);
      int rc = ensure_buf(e, &e->row_ptr, &e->row_ptr_cap, nr * 8, "hipMalloc row_ptr");
      if (rc) return rc;
      // row_ptr now holds these buffers' addresses, not those a plan recorded
      e->rows_src = nullptr;
      e->rows_rep = nullptr;
      e->rows_stride = 0;
      {
        KernelTimer kt(e, NTC_GF256_K_PLAN_ROWS, st, true);
        hipExtLaunchKernelGGL(plan_rows, dim3(static_cast<uint32_t>((nr + 255) / 256)), dim3(256), 0, st,
                           kt.start(), kt.stop(), 0,
                           a.rows_per_gen, a.in_idx, a.G, a.k, a.rows, static_cast<uint64_t>(a.stride),
                           a.in0, a.in1, static_cast<uint64_t*>(e->row_ptr));
      }
      if ((rc = hip_check(hipGetLastError(), "plan_rows launch"))) return rc;
      a.row_ptr = static_cast<const uint64_t*>(e->row_ptr);
    }
  } else {
    const int D = pick_d(a.stride);
    rowtile = 32;
    span = 256u * D;
    wpb = kWaves;
    fn = pick_kernel(dec, D);
  }
  a.nrowchunks = (a.rows + rowtile - 1) / rowtile;
  a.ncolchunks = (a.stride + span - 1) / span;
  a.tile_fast = a.G < 64 ? 1u : 0u;
  uint64_t tasks = static_cast<uint64_t>(a.G) * a.nrowchunks * a.ncolchunks;
  // Split-k: a bit-sliced encode / combine with fewer 16-row tasks than one round of wave slots
  // (3 per SIMD) -- dense n = 1024, G = 1: 2048 -- leaves SIMDs at 2 waves or fewer, each with a
  // long source loop.  Splitting the sources into ksplit parts of >= 64 gives >= 8/3 rounds;
  // the parts' partial repairs are XORed into out afterwards (ksplit_reduce, an HBM pass over
  // ksplit + 1 copies of the output).
  a.ksplit = 1;
  a.kpart = a.k;
  if (span == 2048 && !dec && !a.pair && rowtile == 16) {
    if (!e->ncu) {
      int n = 0;
      if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, e->device) != hipSuccess || n <= 0) n = 256;
      e->ncu = static_cast<uint32_t>(n);
    }
    const uint64_t slots = static_cast<uint64_t>(e->ncu) * 4u * 3u;
    if (tasks < slots && a.k >= 128) {
      // >= 8/3 rounds: measured at n = 1024 (2048 tasks), ksplit 2 / 3 / 4 / 6 / 8 -> MAC 1.01 /
      // 0.93 / 0.90 / 0.93 / 0.90 ms, reduce 0.028 / 0.038 / 0.050 / 0.082 / 0.117 ms per call
      uint32_t ks = static_cast<uint32_t>(std::min<uint64_t>((8 * slots + 3 * tasks - 1) / (3 * tasks), 8));
      if (e->ksplit_force) ks = e->ksplit_force;        // experiments (NTC_GF256_KSPLIT)
      ks = std::min(ks, a.k / 64);
      const uint32_t kpart = (a.k + ks - 1) / ks;
      a.kpart = (kpart + 3) / 4 * 4;
      a.ksplit = (a.k + a.kpart - 1) / a.kpart;          // every part non-empty
    }
  }
  if (a.ksplit > 1) {
    a.kout_step = static_cast<uint64_t>(a.G) * a.rows * a.stride;
    // a stream being captured into a graph must not allocate: without room for the parts, run
    // unsplit (same results; ntc_gf256_reserve cannot size this buffer, it knows no stride)
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if ((a.ksplit - 1) * a.kout_step > e->kout_cap && hipStreamIsCapturing(st, &cap) == hipSuccess &&
        cap != hipStreamCaptureStatusNone) {
      a.ksplit = 1;
      a.kpart = a.k;
    }
  }
  if (a.ksplit > 1 && (a.ksplit - 1) * a.kout_step > e->kout_cap) {
    // the split is an optimisation: without room for the parts the MAC runs unsplit
    void* p = nullptr;
    const size_t na = grow_to(e, (a.ksplit - 1) * a.kout_step, e->kout_cap);
    if (hipMalloc(&p, na) == hipSuccess) {
      drop_buf(e, e->kout);
      e->kout = p;
      e->kout_cap = na;
    } else {
      (void)hipGetLastError();
      a.ksplit = 1;
      a.kpart = a.k;
    }
  }
  if (a.ksplit > 1) {
    a.kout = static_cast<uint8_t*>(e->kout);
    tasks *= a.ksplit;
  }
  if (group > 1) {                              // 4-wave workgroups of 4 / group tile groups
    tasks = tasks / a.nrowchunks * ((a.nrowchunks + group - 1) / group);
    wpb = 4 / group;
  }
  uint32_t threads = group > 1 ? 256 : 64 * wpb;
  if (paired && a.ksplit == 1) {                // one 2-wave workgroup per tile pair
    fn = pick_bsp(dec, a.stride % 2048 == 0, e->pair_j, e->pair_sets);
    tasks = tasks / a.nrowchunks * ((a.nrowchunks + 1) / 2);
    wpb = 1;
    threads = 128;
  }
  const uint64_t blocks = ((tasks + wpb - 1) / wpb + blk_align - 1) / blk_align * blk_align;
  if (blocks > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "batch too large for one launch");
  if (e->timing) (void)hipEventRecord(e->mac_ev[dec][0], st);
  {
    KernelTimer kt(e, dec ? NTC_GF256_K_DECODE_MAC : NTC_GF256_K_ENCODE_MAC, st, true);
    hipExtLaunchKernelGGL(fn, dim3(static_cast<uint32_t>(blocks)), dim3(threads), 0,
                          st, kt.start(), kt.stop(), 0, a);
  }
  int rc = hip_check(hipGetLastError(), what);
  if (!rc && a.ksplit > 1) {
    const uint64_t n16 = a.kout_step / 16;               // stride % 16 == 0
    const uint32_t nblk = static_cast<uint32_t>(std::min<uint64_t>((n16 + 255) / 256, 8192));
    KernelTimer kt(e, NTC_GF256_K_OTHER, st, true);
    hipExtLaunchKernelGGL(ksplit_reduce, dim3(nblk), dim3(256), 0, st, kt.start(), kt.stop(), 0,
                          reinterpret_cast<uint4*>(a.out), reinterpret_cast<const uint4*>(a.kout), n16,
                          a.ksplit - 1);
    rc = hip_check(hipGetLastError(), "ksplit_reduce launch");
  }
  if (e->timing) (void)hipEventRecord(e->mac_ev[dec][1], st);
  return rc;
}

}  // namespace

namespace ntcgpu {

// Coefficient rows padded to the row tile the MAC kernels read (8, 16 or a multiple of 32).
uint32_t tile_rp(uint32_t r)
{
  if (r <= 8) return 8;
  if (r <= 16) return 16;
  return round_up(r, 32);
}

void drop_buf(ntc_gf256_engine* e, void* p)
{
  if (!p) return;
  if (e->captured_any) e->retired.push_back(p);   // a captured graph may still address it
  else (void)hipFree(p);
}

size_t grow_to(const ntc_gf256_engine* e, size_t need, size_t cap)
{
  // after a capture every outgrown buffer is retired, not freed: grow geometrically so that a
  // run of slowly rising shapes retires few of them
  return e->captured_any ? std::max(need, 2 * cap) : need;
}

int ensure_buf(ntc_gf256_engine* e, void** p, size_t* cap, size_t need, const char* what)
{
  if (need <= *cap) return NTC_GPU_OK;
  const size_t n = grow_to(e, need, *cap);
  drop_buf(e, *p);
  *p = nullptr;
  *cap = 0;
  int rc = hip_check(hipMalloc(p, n), what);
  if (rc) return rc;
  *cap = n;
  return NTC_GPU_OK;
}

}  // namespace ntcgpu

namespace {

int ensure_plan(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t rp)
{
  if (G <= e->plan_cap_G && k <= e->plan_cap_k && rp <= e->plan_cap_rp) return NTC_GPU_OK;
  const size_t nG = G > e->plan_cap_G ? grow_to(e, G, e->plan_cap_G) : e->plan_cap_G;
  const size_t nk = k > e->plan_cap_k ? k : e->plan_cap_k;
  const size_t nrp = rp > e->plan_cap_rp ? rp : e->plan_cap_rp;
  (void)hipSetDevice(e->device);
  drop_buf(e, e->plan_m);
  drop_buf(e, e->plan_in);
  drop_buf(e, e->plan_out);
  drop_buf(e, e->plan_coef);
  e->plan_m = nullptr; e->plan_in = nullptr; e->plan_out = nullptr; e->plan_coef = nullptr;
  e->plan_cap_G = e->plan_cap_k = e->plan_cap_rp = 0;
  int rc;
  if ((rc = hip_check(hipMalloc(&e->plan_m, nG * 2), "hipMalloc plan_m"))) return rc;
  if ((rc = hip_check(hipMalloc(&e->plan_in, nG * nk * 2), "hipMalloc plan_in"))) return rc;
  if ((rc = hip_check(hipMalloc(&e->plan_out, nG * nrp * 2), "hipMalloc plan_out"))) return rc;
  if ((rc = hip_check(hipMalloc(&e->plan_coef, nG * nk * nrp + 64), "hipMalloc plan_coef"))) return rc;
  e->plan_cap_G = nG; e->plan_cap_k = nk; e->plan_cap_rp = nrp;
  return NTC_GPU_OK;
}

int check_shape(uint32_t G, uint32_t k, uint32_t r, uint32_t stride)
{
  if (G == 0 || k == 0) return fail(NTC_GPU_EINVAL, "G and k must be > 0");
  if (stride == 0 || stride % 16 != 0) return fail(NTC_GPU_EINVAL, "stride must be a positive multiple of 16");
  if (k > 65535) return fail(NTC_GPU_EUNSUPPORTED, "k > 65535");
  (void)r;
  return NTC_GPU_OK;
}

}  // namespace

extern "C" {

const char* ntc_gf256_last_error(void) { return g_err.c_str(); }

const char* ntc_gf256_build_info(void)
{
  return "libntc_gf256 gfx950: bit-sliced XOR MAC (32 B lanes, 8- or 16-row tiles, one shared "
         "256-block table entered per row with VGPR-relative accumulators) for strides filling >= "
         "1/3 of a 2 KiB wave span; v_perm_b32 3/3/2 split MAC (R in {4,8,16,32}, D in {1,2}) "
         "otherwise";
}

uint32_t ntc_gf256_coefficient(uint32_t repair_id, uint32_t src_id) { return coefficient(repair_id, src_id); }

uint16_t ntc_gf256_multiply_size(uint16_t size, uint32_t coeff)
{
  if (size == 0 || coeff == 0) return 0;
  const uint8_t c = static_cast<uint8_t>(coeff);
  return static_cast<uint16_t>(field_mul(c, size & 0xFF) | (field_mul(c, size >> 8) << 8));
}

uint8_t ntc_gf256_multiply(uint8_t x, uint8_t y) { return field_mul(x, y); }
uint8_t ntc_gf256_invert(uint8_t x) { return x ? field_inv(x) : 0; }

int ntc_gf256_engine_create(int device, ntc_gf256_engine** out)
{
  if (!out) return fail(NTC_GPU_EINVAL, "out is NULL");
  *out = nullptr;
  int n = 0;
  int rc = hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (rc) return rc;
  if (device < 0 || device >= n) return fail(NTC_GPU_EINVAL, "no such HIP device");
  if ((rc = hip_check(hipSetDevice(device), "hipSetDevice"))) return rc;
  hipDeviceProp_t prop;
  if ((rc = hip_check(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties"))) return rc;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(NTC_GPU_EUNSUPPORTED, std::string("built for gfx950, device is ") + prop.gcnArchName);
  auto* e = new (std::nothrow) ntc_gf256_engine;
  if (!e) return fail(NTC_GPU_ENOMEM, "host allocation");
  e->device = device;
  // process-wide overrides of the AUTO choices (gpu.h): A/B runs without a rebuild
  if (const char* m = std::getenv("NTC_GF256_MAC")) {
    if (!std::strcmp(m, "perm")) e->mac_kind = NTC_GF256_MAC_PERM;
    else if (!std::strcmp(m, "bitslice")) e->mac_kind = NTC_GF256_MAC_BITSLICE;
    else if (!std::strcmp(m, "grouped")) e->mac_kind = NTC_GF256_MAC_BITSLICE_GROUPED;
    else if (!std::strcmp(m, "paired")) e->mac_kind = NTC_GF256_MAC_BITSLICE_PAIRED;
  }
  if (const char* t = std::getenv("NTC_GF256_PAIRJ")) {
    if (!std::strcmp(t, "1")) e->pair_j = 1;
    else if (!std::strcmp(t, "2")) e->pair_j = 2;
  }
  if (const char* t = std::getenv("NTC_GF256_PAIRSETS")) {
    if (!std::strcmp(t, "3")) e->pair_sets = 3;
    else if (!std::strcmp(t, "4")) e->pair_sets = 4;
  }
  if (const char* t = std::getenv("NTC_GF256_KSPLIT")) {
    const int v = std::atoi(t);
    if (v >= 1 && v <= 8) e->ksplit_force = static_cast<uint32_t>(v);
  }
  if (const char* t = std::getenv("NTC_GF256_SLICE")) {
    if (!std::strcmp(t, "0")) e->slice_force = 0;
    else if (!std::strcmp(t, "1")) e->slice_force = 1;
  }
  if (const char* t = std::getenv("NTC_GF256_ROWTILE")) {
    if (!std::strcmp(t, "8")) e->rowtile_force = 8;
    else if (!std::strcmp(t, "16")) e->rowtile_force = 16;
  }
  if (const char* p = std::getenv("NTC_GF256_PLAN")) {
    if (!std::strcmp(p, "wave")) e->plan_kind = NTC_GF256_PLAN_WAVE;
    else if (!std::strcmp(p, "lds")) e->plan_kind = NTC_GF256_PLAN_LDS;
    else if (!std::strcmp(p, "big")) e->plan_kind = NTC_GF256_PLAN_BIG;
  }
  *out = e;
  return NTC_GPU_OK;
}

void ntc_gf256_engine_destroy(ntc_gf256_engine* e)
{
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipFree(e->plan_m);
  (void)hipFree(e->plan_in);
  (void)hipFree(e->plan_out);
  (void)hipFree(e->plan_coef);
  (void)hipFree(e->enc_coef);
  (void)hipFree(e->enc_pair);
  (void)hipFree(e->kout);
  (void)hipFree(e->slice);
  (void)hipFree(e->row_ptr);
  for (void* b : {e->dn_x, e->dn_y, e->dn_w, e->dn_piv, e->dn_flag, e->dn_coef, e->dn_ok}) (void)hipFree(b);
  for (void* b : e->retired) (void)hipFree(b);
  for (auto& pair : e->mac_ev)
    for (hipEvent_t ev : pair)
      if (ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : e->tlog_ev)
    if (ev) (void)hipEventDestroy(ev);
  delete e;
}

int ntc_gf256_set_timing(ntc_gf256_engine* e, int on)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  (void)hipSetDevice(e->device);
  for (auto& pair : e->mac_ev)
    for (hipEvent_t& ev : pair)
      if (!ev) {
        int rc = hip_check(hipEventCreate(&ev), "hipEventCreate");
        if (rc) return rc;
      }
  e->timing = on != 0;
  return NTC_GPU_OK;
}

int ntc_gf256_mac_time(ntc_gf256_engine* e, int dec, float* ms)
{
  if (!e || !ms) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (!e->timing) return fail(NTC_GPU_EINVAL, "timing is off (ntc_gf256_set_timing)");
  hipEvent_t* ev = e->mac_ev[dec ? 1 : 0];
  int rc = hip_check(hipEventSynchronize(ev[1]), "hipEventSynchronize");
  if (rc) return rc;
  return hip_check(hipEventElapsedTime(ms, ev[0], ev[1]), "hipEventElapsedTime");
}

int ntc_gf256_set_mac_kind(ntc_gf256_engine* e, int kind)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  if (kind < NTC_GF256_MAC_AUTO || kind > NTC_GF256_MAC_BITSLICE_PAIRED) return fail(NTC_GPU_EINVAL, "unknown MAC kind");
  e->mac_kind = kind;
  return NTC_GPU_OK;
}

int ntc_gf256_release_retired(ntc_gf256_engine* e)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  (void)hipSetDevice(e->device);
  for (void* b : e->retired) (void)hipFree(b);
  e->retired.clear();
  return NTC_GPU_OK;
}

int ntc_gf256_set_plan_kind(ntc_gf256_engine* e, int kind)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  if (kind < NTC_GF256_PLAN_AUTO || kind > NTC_GF256_PLAN_BIG) return fail(NTC_GPU_EINVAL, "unknown plan kind");
  e->plan_kind = kind;
  return NTC_GPU_OK;
}

int ntc_gf256_timing_log(ntc_gf256_engine* e, uint32_t capacity)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  (void)hipSetDevice(e->device);
  // events of a previous log may still be pending on some stream: wait before reusing them
  for (uint32_t i = 0; i < e->tlog_n; ++i) (void)hipEventSynchronize(e->tlog_ev[2 * i + 1]);
  e->tlog_n = 0;
  e->tlog_cap = 0;
  if (2u * capacity > e->tlog_ev.size()) {
    const size_t have = e->tlog_ev.size();
    e->tlog_ev.resize(2u * capacity, nullptr);
    for (size_t i = have; i < e->tlog_ev.size(); ++i) {
      int rc = hip_check(hipEventCreate(&e->tlog_ev[i]), "hipEventCreate");
      if (rc) {
        e->tlog_ev.resize(i);
        return rc;
      }
    }
  }
  e->tlog_kind.assign(capacity, NTC_GF256_K_OTHER);
  e->tlog_cap = capacity;
  return NTC_GPU_OK;
}

int ntc_gf256_timing_kinds(ntc_gf256_engine* e, uint32_t mask)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  e->tlog_mask = mask;
  return NTC_GPU_OK;
}

int ntc_gf256_timing_read(ntc_gf256_engine* e, uint32_t max, uint32_t* n, uint32_t* kinds, float* ms)
{
  if (!e || !n || (max && (!kinds || !ms))) return fail(NTC_GPU_EINVAL, "NULL argument");
  *n = e->tlog_n;
  const uint32_t cnt = e->tlog_n < max ? e->tlog_n : max;
  for (uint32_t i = 0; i < cnt; ++i) {
    int rc = hip_check(hipEventSynchronize(e->tlog_ev[2 * i + 1]), "hipEventSynchronize");
    if (rc) return rc;
    if ((rc = hip_check(hipEventElapsedTime(&ms[i], e->tlog_ev[2 * i], e->tlog_ev[2 * i + 1]),
                        "hipEventElapsedTime")))
      return rc;
    kinds[i] = e->tlog_kind[i];
  }
  return NTC_GPU_OK;
}

int ntc_gf256_reserve(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  (void)hipSetDevice(e->device);
  const uint32_t rp = tile_rp(r);
  int rc = ensure_buf(e, &e->enc_coef, &e->enc_coef_cap, static_cast<size_t>(G) * k * rp + 64, "hipMalloc enc_coef");
  if (rc) return rc;
  if ((rc = ensure_buf(e, &e->enc_pair, &e->enc_pair_cap, G, "hipMalloc enc_pair"))) return rc;
  // the decode MAC's input row addresses (decode_plan_w / plan_rows), so later calls never allocate
  if ((rc = ensure_buf(e, &e->row_ptr, &e->row_ptr_cap, static_cast<size_t>(G) * (k + kBsRing) * 8,
                       "hipMalloc row_ptr")))
    return rc;
  return ensure_plan(e, G, k, rp);
}

int ntc_gf256_encode_batch(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                           uint32_t stride, const uint8_t* src, const uint16_t* src_len,
                           const uint32_t* sid_base, const uint32_t* rid_base, uint8_t* rep,
                           uint16_t* rep_size, uint16_t* rep_len, void* stream)
{
  if (!e || !src || !src_len || !rep || !rep_size) return fail(NTC_GPU_EINVAL, "NULL argument");
  int rc = check_shape(G, k, r, stride);
  if (rc) return rc;
  if (r == 0) return NTC_GPU_OK;
  (void)hipSetDevice(e->device);
  const uint32_t rp = tile_rp(r);
  hipStream_t st = static_cast<hipStream_t>(stream);
  rc = ensure_buf(e, &e->enc_coef, &e->enc_coef_cap, static_cast<size_t>(G) * k * rp + 64, "hipMalloc enc_coef");
  if (rc) return rc;
  // generation pairing (kPairGap): symbols of at most half a bit-sliced span that fill at least a
  // third of it when paired; pays off with continuous ids.  Under AUTO, a stride the unpaired
  // bit-sliced kernel would not take (< 1/3 of a span) pairs only with the default continuous
  // ids: explicit id bases may leave every generation unpaired, and an unpaired PAIR wave runs
  // half its lanes idle where the v_perm MAC would have been chosen.
  const bool pairing = G > kPairGap && stride <= 1024 &&
                       (e->mac_kind == NTC_GF256_MAC_BITSLICE ||
                        (e->mac_kind == NTC_GF256_MAC_AUTO && 2u * stride * 100u >= 2048u * 33u &&
                         (use_bitslice(e, stride) || (!sid_base && !rid_base))));
  if (pairing &&
      (rc = ensure_buf(e, &e->enc_pair, &e->enc_pair_cap, G, "hipMalloc enc_pair")))
    return rc;
  PrepArgs p{};
  p.G = G; p.k = k; p.r = r; p.rp = rp; p.src_len = src_len; p.sid_base = sid_base;
  p.rid_base = rid_base; p.rep_size = rep_size; p.rep_len = rep_len;
  p.coef = static_cast<uint8_t*>(e->enc_coef);
  p.pair = pairing ? static_cast<uint8_t*>(e->enc_pair) : nullptr;
  {
    KernelTimer kt(e, NTC_GF256_K_ENCODE_PREP, st, true);
    hipExtLaunchKernelGGL(encode_prep, dim3((G + 3) / 4), dim3(256), 0, st, kt.start(), kt.stop(), 0, p);
  }
  if ((rc = hip_check(hipGetLastError(), "encode_prep launch"))) return rc;
  MacArgs a{};
  a.G = G; a.k = k; a.rows = r; a.stride = stride;
  a.in0 = src; a.out = rep; a.coef = static_cast<const uint8_t*>(e->enc_coef); a.rp = rp;
  a.pair = p.pair;
  a.pair_in = static_cast<uint64_t>(kPairGap) * k * stride;
  a.pair_out = static_cast<uint64_t>(kPairGap) * r * stride;
  return launch_mac(e, false, a, st, "encode_mac launch");
}

// rows_src / rows_rep (decode_batch, which knows the apply's buffers): a register plan also
// writes the decode MAC's input row addresses, so the apply skips plan_rows.
static int plan_impl(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r, uint16_t* src_len,
                     const uint8_t* src_mask, const uint16_t* rep_size, const uint8_t* rep_mask,
                     const uint32_t* sid_base, const uint32_t* rid_base,
                     ntc_gf256_decode_status* status, void* stream,
                     const uint8_t* rows_src = nullptr, const uint8_t* rows_rep = nullptr,
                     uint32_t rows_stride = 0)
{
  if (!e || !src_len || !src_mask || !rep_size || !rep_mask || !status)
    return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0) return fail(NTC_GPU_EINVAL, "G and k must be > 0");
  if (r > kBigRows) return fail(NTC_GPU_EUNSUPPORTED, "r > 255 not supported by decode (w = 8 limit)");
  if (k > 65535) return fail(NTC_GPU_EUNSUPPORTED, "k > 65535");
  // plan kernel: the engine's plan kind (ntc_gf256_set_plan_kind; results are identical)
  const int kind = e->plan_kind;
  const bool big = r > static_cast<uint32_t>(kMaxPlanRows) || (kind == NTC_GF256_PLAN_BIG && r > 0);
  const uint32_t rp = tile_rp(r);
  (void)hipSetDevice(e->device);
  int rc = ensure_plan(e, G, k, rp);
  if (rc) return rc;
  PlanArgs p{};
  p.G = G; p.k = k; p.r = r; p.src_len = src_len; p.src_mask = src_mask; p.rep_size = rep_size;
  p.rep_mask = rep_mask; p.sid_base = sid_base; p.rid_base = rid_base; p.status = status;
  p.plan_m = e->plan_m; p.plan_in = e->plan_in; p.plan_out = e->plan_out;
  p.plan_coef = e->plan_coef; p.rp = rp;
  // r <= 32: the register-resident plan (four generations per block); PLAN_LDS selects the LDS
  // Gauss-Jordan kernel instead (r > 32 always uses it)
  const bool lds_plan = kind == NTC_GF256_PLAN_LDS;
  const bool wave_plan = !big && r <= 32 && !lds_plan;
  if (wave_plan && rows_src && rows_rep && use_bitslice(e, rows_stride)) {
    rc = ensure_buf(e, &e->row_ptr, &e->row_ptr_cap, static_cast<uint64_t>(G) * (k + kBsRing) * 8,
                    "hipMalloc row_ptr");
    if (rc) return rc;
    p.rows_out = static_cast<uint64_t*>(e->row_ptr);
    p.rows_src = rows_src;
    p.rows_rep = rows_rep;
    p.rows_stride = rows_stride;
  }
  if (big) {
    static const int lds_ok = [] {
      return static_cast<int>(hipFuncSetAttribute(reinterpret_cast<const void*>(decode_plan_big),
                                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                                  static_cast<int>(big_lds_bytes(260, 129, 256))));
    }();
    if (lds_ok != 0) return fail(NTC_GPU_EDEVICE, "decode_plan_big: LDS attribute");
  }
  // the plan is one launch (a timed ext launch) except the large-window path's two
  KernelTimer kt(e, NTC_GF256_K_DECODE_PLAN, static_cast<hipStream_t>(stream), !big);
  if (big) {
    // matrix rows of 2 * mmax bytes (odd dword pitch), r rows padded so ptab stays 16-B aligned
    auto launch_big = [&](uint32_t mmax, uint32_t cap, uint32_t deferred) {
      p.big_pitch = ((2 * mmax + 3) / 4) | 1u;
      p.big_rows = r;
      while ((p.big_rows * p.big_pitch) % 4u) ++p.big_rows;
      p.m_cap = cap;
      p.deferred_only = deferred;
      hipLaunchKernelGGL(decode_plan_big, dim3(G), dim3(256), big_lds_bytes(p.big_rows, p.big_pitch, mmax),
                         static_cast<hipStream_t>(stream), p);
    };
    if (r > kBigCap) {
      launch_big(kBigCap, kBigCap, 0);          // every generation with m <= kBigCap
      launch_big(r, 0, 1);                      // the deferred ones, full-size rows
    } else {
      launch_big(r, 0, 0);
    }
  } else if (wave_plan) {
    auto* fw = r <= 8 ? decode_plan_w<8> : r <= 16 ? decode_plan_w<16> : decode_plan_w<32>;
    hipExtLaunchKernelGGL(fw, dim3((G + kPlanWaves - 1) / kPlanWaves), dim3(64 * kPlanWaves), 0,
                          static_cast<hipStream_t>(stream), kt.start(), kt.stop(), 0, p);
  } else {
    auto* fn = r <= 8 ? decode_plan<8> : r <= 16 ? decode_plan<16> : r <= 32 ? decode_plan<32> : decode_plan<64>;
    hipExtLaunchKernelGGL(fn, dim3(G), dim3(64), 0, static_cast<hipStream_t>(stream), kt.start(),
                          kt.stop(), 0, p);
  }
  e->last_G = G; e->last_k = k; e->last_r = r; e->last_rp = rp;
  e->rows_src = p.rows_out ? rows_src : nullptr;
  e->rows_rep = p.rows_out ? rows_rep : nullptr;
  e->rows_stride = p.rows_out ? rows_stride : 0;
  return hip_check(hipGetLastError(), "decode_plan launch");
}

int ntc_gf256_decode_plan(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                          uint16_t* src_len, const uint8_t* src_mask, const uint16_t* rep_size,
                          const uint8_t* rep_mask, const uint32_t* sid_base,
                          const uint32_t* rid_base, ntc_gf256_decode_status* status, void* stream)
{
  return plan_impl(e, G, k, r, src_len, src_mask, rep_size, rep_mask, sid_base, rid_base, status,
                   stream);
}

int ntc_gf256_decode_apply(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                           uint32_t stride, uint8_t* src, const uint8_t* rep, void* stream)
{
  if (!e || !src || !rep) return fail(NTC_GPU_EINVAL, "NULL argument");
  int rc = check_shape(G, k, r, stride);
  if (rc) return rc;
  if (G != e->last_G || k != e->last_k || r != e->last_r)
    return fail(NTC_GPU_EINVAL, "decode_apply geometry differs from the last decode_plan");
  if (r == 0) return NTC_GPU_OK;
  MacArgs a{};
  a.G = G; a.k = k; a.rows = r; a.stride = stride;
  a.in0 = src; a.in1 = rep; a.out = src;
  a.rows_per_gen = e->plan_m; a.in_idx = e->plan_in; a.out_idx = e->plan_out;
  a.coef = e->plan_coef; a.rp = e->last_rp;
  // row addresses already written by the plan for exactly these buffers (launch_mac forgets them
  // whenever plan_rows overwrites row_ptr for other buffers)
  if (e->rows_src == src && e->rows_rep == rep && e->rows_stride == stride && src)
    a.row_ptr = static_cast<const uint64_t*>(e->row_ptr);
  return launch_mac(e, true, a, static_cast<hipStream_t>(stream), "decode_mac launch");
}

int ntc_gf256_decode_batch(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                           uint32_t stride, uint8_t* src, uint16_t* src_len,
                           const uint8_t* src_mask, const uint8_t* rep, const uint16_t* rep_size,
                           const uint8_t* rep_mask, const uint32_t* sid_base,
                           const uint32_t* rid_base, ntc_gf256_decode_status* status, void* stream)
{
  int rc = check_shape(G, k, r, stride);
  if (rc) return rc;
  // the register plan also writes the bit-sliced decode MAC's input row addresses
  rc = plan_impl(e, G, k, r, src_len, src_mask, rep_size, rep_mask, sid_base, rid_base, status,
                 stream, src, rep, stride);
  if (rc) return rc;
  return ntc_gf256_decode_apply(e, G, k, r, stride, src, rep, stream);
}

uint32_t ntc_gf256_coef_pitch(uint32_t rows) { return tile_rp(rows); }

int ntc_gf256_combine_batch(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t rows,
                            uint32_t stride, const uint8_t* in, const uint8_t* coef, uint8_t* out,
                            void* stream)
{
  if (!e || !in || !coef || !out) return fail(NTC_GPU_EINVAL, "NULL argument");
  int rc = check_shape(G, k, rows, stride);
  if (rc) return rc;
  if (rows == 0) return NTC_GPU_OK;
  MacArgs a{};
  a.G = G; a.k = k; a.rows = rows; a.stride = stride;
  a.in0 = in; a.out = out; a.coef = coef; a.rp = tile_rp(rows);
  return launch_mac(e, false, a, static_cast<hipStream_t>(stream), "combine launch");
}

int ntc_gf256_gather_combine(ntc_gf256_engine* e, uint32_t njobs, const ntc_gf256_gather_job* jobs,
                             const ntc_gf256_gather_term* terms, uint32_t max_len, void* stream)
{
  if (!e || (njobs && (!jobs || !terms))) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (njobs == 0 || max_len == 0) return NTC_GPU_OK;
  if (max_len > 65535) return fail(NTC_GPU_EUNSUPPORTED, "gather_combine: payloads up to 65535 bytes");
  (void)hipSetDevice(e->device);
  hipLaunchKernelGGL(gather_combine, dim3(njobs, (max_len + 1023) / 1024), dim3(64), 0,
                     static_cast<hipStream_t>(stream), jobs, terms);
  return hip_check(hipGetLastError(), "gather_combine launch");
}

int ntc_gf256_region_multiply(ntc_gf256_engine* e, const uint8_t* src, uint8_t* dst, size_t len,
                              uint8_t c, int add, void* stream)
{
  if (!e || (!src && len) || (!dst && len)) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (len == 0) return NTC_GPU_OK;
  size_t blocks = (len / 4 + 255) / 256;
  if (blocks == 0) blocks = 1;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(region_mul, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), src, dst, len, static_cast<uint32_t>(c), add);
  return hip_check(hipGetLastError(), "region_mul launch");
}

}  // extern "C"
