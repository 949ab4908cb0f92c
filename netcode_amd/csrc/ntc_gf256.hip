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

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gf256_field.hh"
#include "netcode/gpu.h"

namespace ntcgpu {

__constant__ PermTables d_perm = make_perm_tables();
__constant__ FieldTables d_field = make_field_tables();

constexpr int kWaves = 4;               // waves per 256-thread block
constexpr int kMaxPlanRows = 64;        // m <= 64 (r <= 64) in this build

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
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
};

// One wave computes R output rows x (64 lanes x 4D bytes) of one generation:
//   out[row] = sum_i coef[i][row] * in[i]
// Inputs are consumed in pairs with the next pair's loads in flight (register double buffer).
template <int R, int D, bool DEC>
__device__ __forceinline__ void mac_tile(const MacArgs& a, uint32_t g, uint32_t row0, uint32_t nrows,
                                         uint32_t col, bool active)
{
  const size_t stride = a.stride;
  const uint32_t k = a.k;
  const uint32_t colx = active ? col : 0u;
  const uint8_t* base0 = a.in0 + static_cast<size_t>(g) * k * stride + colx;
  const uint8_t* base1 = DEC ? a.in1 + static_cast<size_t>(g) * a.rows * stride + colx : nullptr;
  const uint16_t* in = DEC ? a.in_idx + static_cast<size_t>(g) * k : nullptr;
  const uint8_t* coef = a.coef + static_cast<size_t>(g) * k * a.rp + row0;
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
  uint32_t n0[D], n1[D];
  if (kk) {
    load_row<D>(rowptr(0), n0);
    load_row<D>(rowptr(1), n1);
  }
  for (uint32_t i = 0; i < kk; i += 2) {
    uint32_t x0[D], x1[D];
#pragma unroll
    for (int d = 0; d < D; ++d) { x0[d] = n0[d]; x1[d] = n1[d]; }
    if (i + 2 < kk) {
      load_row<D>(rowptr(i + 2), n0);
      load_row<D>(rowptr(i + 3), n1);
    }
    Sel<D> s0, s1;
    s0.make(x0);
    s1.make(x1);
    const uint32_t* cw0 = reinterpret_cast<const uint32_t*>(coef + i * a.rp);
    const uint32_t* cw1 = reinterpret_cast<const uint32_t*>(coef + (i + 1) * a.rp);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint32_t c0 = (cw0[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      const uint32_t c1 = (cw1[j >> 2] >> (8 * (j & 3))) & 0xFFu;
      mac2<D>(acc[j], c0, s0, c1, s1);
    }
  }
  if (k & 1u) {
    uint32_t x0[D];
    load_row<D>(rowptr(kk), x0);
    Sel<D> s0;
    s0.make(x0);
    const uint32_t* cw0 = reinterpret_cast<const uint32_t*>(coef + kk * a.rp);
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
  const uint32_t total = DEC ? uniform(a.rows_per_gen[g]) : a.rows;
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
struct PrepArgs {
  uint32_t G, k, r, rp;
  const uint16_t* src_len;
  const uint32_t* sid_base;
  const uint32_t* rid_base;
  uint8_t* coef;
  uint16_t* rep_size;
  uint16_t* rep_len;
};

__global__ __launch_bounds__(256) void encode_prep(PrepArgs a)
{
  const uint32_t g = blockIdx.x;
  const uint32_t sidb = a.sid_base ? a.sid_base[g] : g * a.k;
  const uint32_t ridb = a.rid_base ? a.rid_base[g] : g * a.r;
  uint8_t* coef = a.coef + static_cast<size_t>(g) * a.k * a.rp;
  const uint32_t n = a.k * a.rp;
  for (uint32_t t = threadIdx.x * 4; t < n; t += 256 * 4) {
    uint32_t w = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
      const uint32_t i = (t + b) / a.rp, j = (t + b) % a.rp;
      if (j < a.r) w |= coefficient(ridb + j, sidb + i) << (8 * b);
    }
    *reinterpret_cast<uint32_t*>(coef + t) = w;   // rp is a multiple of 4
  }
  const uint16_t* len = a.src_len + static_cast<size_t>(g) * a.k;
  for (uint32_t j = threadIdx.x; j < a.r; j += 256) {
    uint16_t esz = 0;
    for (uint32_t i = 0; i < a.k; ++i)
      esz ^= mul_size(len[i], static_cast<uint8_t>(coefficient(ridb + j, sidb + i)));
    a.rep_size[static_cast<size_t>(g) * a.r + j] = esz;
  }
  if (a.rep_len && threadIdx.x < 64) {
    uint32_t mx = 0;
    for (uint32_t t = threadIdx.x; t < a.k; t += 64) mx = max(mx, static_cast<uint32_t>(len[t]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, o)));
    if (threadIdx.x == 0) a.rep_len[g] = static_cast<uint16_t>(mx);
  }
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
};

__global__ __launch_bounds__(64) void decode_plan(PlanArgs a)
{
  __shared__ uint8_t exp_t[512];
  __shared__ uint8_t log_t[256];
  __shared__ uint8_t A[kMaxPlanRows][2 * kMaxPlanRows + 4];
  __shared__ uint16_t miss[kMaxPlanRows];
  __shared__ uint16_t recv[kMaxPlanRows];
  __shared__ uint16_t reps[kMaxPlanRows];
  __shared__ uint32_t sizes[kMaxPlanRows];
  __shared__ uint8_t dacc[64][kMaxPlanRows + 4];

  const uint32_t lane = threadIdx.x;
  const uint32_t g = blockIdx.x;
  for (uint32_t t = lane; t < 512; t += 64) exp_t[t] = d_field.exp[t];
  for (uint32_t t = lane; t < 256; t += 64) log_t[t] = d_field.log[t];
  __syncthreads();
  auto mul = [&](uint32_t x, uint32_t y) -> uint32_t {
    return (x == 0 || y == 0) ? 0u : exp_t[log_t[x] + log_t[y]];
  };

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
      if (pos < kMaxPlanRows) miss[pos] = static_cast<uint16_t>(idx);
    }
    m += __popcll(b);
  }
  uint32_t nrecv = 0;
  for (uint32_t base = 0; base < r; base += 64) {
    const uint32_t idx = base + lane;
    const bool got = idx < r && rmask[idx] != 0;
    const uint64_t b = __ballot(got);
    if (got) {
      const uint32_t pos = nrecv + __popcll(b & lt);
      if (pos < kMaxPlanRows) recv[pos] = static_cast<uint16_t>(idx);
    }
    nrecv += __popcll(b);
  }
  __syncthreads();

  ntc_gf256_decode_status st{};
  st.nb_missing = static_cast<uint16_t>(m);
  st.last_repair = 0xFFFF;
  uint32_t mm = 0;  // rows of the decode matrix written to the plan

  if (m == 0) {
    st.state = 1;
    st.nb_useless = static_cast<uint16_t>(nrecv);
  } else if (nrecv < m || m > kMaxPlanRows) {
    st.state = 2;
  } else {
    bool ok = false;
    uint32_t t = m - 1;
    for (; t < nrecv; ++t) {
      for (uint32_t q = lane; q < m; q += 64) reps[q] = (q + 1 < m) ? recv[q] : recv[t];
      __syncthreads();
      // A[q][c]: storage row q = repair q (the reference's column-major square_matrix), columns
      // 0..m-1 = coefficient of missing source c, m..2m-1 = identity.
      for (uint32_t q = 0; q < m; ++q) {
        const uint32_t rid = ridb + reps[q];
        for (uint32_t c = lane; c < 2 * m; c += 64) {
          A[q][c] = (c < m) ? static_cast<uint8_t>(coefficient(rid, sidb + miss[c]))
                            : static_cast<uint8_t>((c - m) == q ? 1 : 0);
        }
      }
      __syncthreads();
      bool singular = false;
      for (uint32_t p = 0; p < m; ++p) {
        const bool cand = lane >= p && lane < m && A[lane][p] != 0;
        const uint64_t b = __ballot(cand);
        if (b == 0) { singular = true; break; }
        const uint32_t q = __ffsll(static_cast<unsigned long long>(b)) - 1;
        if (q != p) {
          for (uint32_t c = lane; c < 2 * m; c += 64) {
            const uint8_t tmp = A[p][c];
            A[p][c] = A[q][c];
            A[q][c] = tmp;
          }
        }
        __syncthreads();
        const uint32_t inv = exp_t[(255 - log_t[A[p][p]]) % 255];
        for (uint32_t c = lane; c < 2 * m; c += 64) A[p][c] = static_cast<uint8_t>(mul(A[p][c], inv));
        __syncthreads();
        for (uint32_t q2 = 0; q2 < m; ++q2) {
          if (q2 == p) continue;
          const uint32_t f = A[q2][p];
          __syncthreads();
          if (f != 0)
            for (uint32_t c = lane; c < 2 * m; c += 64) A[q2][c] ^= static_cast<uint8_t>(mul(f, A[p][c]));
          __syncthreads();
        }
      }
      if (!singular) { ok = true; break; }
      __syncthreads();
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
      // Input list: positions 0..m-1 = the chosen repairs, m..k-1 = received sources ascending.
      uint16_t* pin = a.plan_in + static_cast<size_t>(g) * k;
      uint8_t* pc = a.plan_coef + static_cast<size_t>(g) * k * a.rp;
      uint16_t* pout = a.plan_out + static_cast<size_t>(g) * a.rp;
      for (uint32_t s = lane; s < a.rp; s += 64) pout[s] = (s < m) ? miss[s] : 0;
      for (uint32_t s = lane; s < m; s += 64) sizes[s] = 0;
      __syncthreads();
      const uint16_t* rsz = a.rep_size + static_cast<size_t>(g) * r;
      const uint16_t* slen = a.src_len + static_cast<size_t>(g) * k;
      for (uint32_t q = 0; q < m; ++q) {
        if (lane == 0) pin[q] = static_cast<uint16_t>(k + reps[q]);
        const uint16_t val = rsz[reps[q]];
        for (uint32_t s = lane; s < a.rp; s += 64) {
          const uint32_t dsq = (s < m) ? A[s][m + q] : 0u;   // (M^-1)[s][q]
          pc[static_cast<size_t>(q) * a.rp + s] = static_cast<uint8_t>(dsq);
          if (s < m) sizes[s] ^= mul_size(val, static_cast<uint8_t>(dsq));
        }
      }
      __syncthreads();
      // Received sources: D[s][j] = sum_q (M^-1)[s][q] * c(rep_q, j); one source per lane,
      // the lane's column accumulated in LDS (dacc[lane][s]).
      uint32_t pos_base = m;
      for (uint32_t base = 0; base < k; base += 64) {
        const uint32_t j = base + lane;
        const bool got = j < k && smask[j] != 0;
        const uint64_t b = __ballot(got);
        if (got) {
          const uint32_t pos = pos_base + __popcll(b & lt);
          pin[pos] = static_cast<uint16_t>(j);
          const uint16_t val = slen[j];
          for (uint32_t s = 0; s < m; ++s) dacc[lane][s] = 0;
          for (uint32_t q = 0; q < m; ++q) {
            const uint32_t lc = log_t[coefficient(ridb + reps[q], sidb + j)];
            for (uint32_t s = 0; s < m; ++s) {
              const uint32_t x = A[s][m + q];
              if (x) dacc[lane][s] ^= exp_t[log_t[x] + lc];
            }
          }
          uint8_t* col = pc + static_cast<size_t>(pos) * a.rp;
          for (uint32_t s = 0; s < a.rp; ++s) {
            const uint32_t dsj = (s < m) ? dacc[lane][s] : 0u;
            col[s] = static_cast<uint8_t>(dsj);
            if (s < m) atomicXor(&sizes[s], static_cast<uint32_t>(mul_size(val, static_cast<uint8_t>(dsj))));
          }
        }
        pos_base += __popcll(b);
      }
      __syncthreads();
      uint16_t* olen = a.src_len + static_cast<size_t>(g) * k;
      for (uint32_t s = lane; s < m; s += 64) olen[miss[s]] = static_cast<uint16_t>(sizes[s]);
    }
  }
  if (lane == 0) {
    a.plan_m[g] = static_cast<uint16_t>(mm);
    a.status[g] = st;
  }
}

// ----------------------------------------------------------------------- region multiply ----
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

struct ntc_gf256_engine {
  int device = 0;
  size_t plan_cap_G = 0, plan_cap_k = 0, plan_cap_rp = 0;
  uint16_t* plan_m = nullptr;
  uint16_t* plan_in = nullptr;
  uint16_t* plan_out = nullptr;
  uint8_t* plan_coef = nullptr;
  void* enc_coef = nullptr;
  size_t enc_coef_cap = 0;
  // geometry of the last plan (decode_apply must match)
  uint32_t last_G = 0, last_k = 0, last_r = 0, last_rp = 0;
};

namespace {

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

uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

// Column width per lane: widest that still fills most lanes of the last column chunk.
int pick_d(uint32_t stride)
{
  // NTC_GF256_FORCE_D=1|2|4 overrides the choice (tuning experiments only).
  static const int forced = [] {
    const char* v = std::getenv("NTC_GF256_FORCE_D");
    return v ? std::atoi(v) : 0;
  }();
  if ((forced == 1 || forced == 2 || forced == 4) && stride % (4u * forced) == 0) return forced;
  // Prefer 16 B per lane (dwordx4) unless the last column chunk would leave >10 % of lanes idle.
  for (int D = 4; D >= 2; D /= 2) {
    const uint32_t span = 256u * D;
    const uint32_t chunks = (stride + span - 1) / span;
    if (stride % (4u * D) == 0 && 10ull * stride >= 9ull * chunks * span) return D;
  }
  return stride % 8 == 0 && stride >= 512 ? 2 : 1;
}

typedef void (*mac_fn)(MacArgs);

mac_fn pick_kernel(bool dec, int D)
{
  if (dec) return D == 4 ? gf_mac<4, true> : D == 2 ? gf_mac<2, true> : gf_mac<1, true>;
  return D == 4 ? gf_mac<4, false> : D == 2 ? gf_mac<2, false> : gf_mac<1, false>;
}

// Coefficient rows padded to the row tile the MAC kernel reads (4, 8, 16 or a multiple of 32).
uint32_t tile_rp(uint32_t r)
{
  if (r <= 4) return 4;
  if (r <= 8) return 8;
  if (r <= 16) return 16;
  return round_up(r, 32);
}

int ensure_buf(void** p, size_t* cap, size_t need, const char* what)
{
  if (need <= *cap) return NTC_GPU_OK;
  (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  int rc = hip_check(hipMalloc(p, need), what);
  if (rc) return rc;
  *cap = need;
  return NTC_GPU_OK;
}

int ensure_plan(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t rp)
{
  if (G <= e->plan_cap_G && k <= e->plan_cap_k && rp <= e->plan_cap_rp) return NTC_GPU_OK;
  const size_t nG = G > e->plan_cap_G ? G : e->plan_cap_G;
  const size_t nk = k > e->plan_cap_k ? k : e->plan_cap_k;
  const size_t nrp = rp > e->plan_cap_rp ? rp : e->plan_cap_rp;
  (void)hipSetDevice(e->device);
  (void)hipFree(e->plan_m);
  (void)hipFree(e->plan_in);
  (void)hipFree(e->plan_out);
  (void)hipFree(e->plan_coef);
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
  return "libntc_gf256 gfx950: v_perm_b32 3/3/2 split + v_bitop3 XOR, R in {4,8,16,32}, D in {1,2,4}";
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
  delete e;
}

int ntc_gf256_reserve(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r)
{
  if (!e) return fail(NTC_GPU_EINVAL, "engine is NULL");
  (void)hipSetDevice(e->device);
  const uint32_t rp = tile_rp(r);
  int rc = ensure_buf(&e->enc_coef, &e->enc_coef_cap, static_cast<size_t>(G) * k * rp + 64, "hipMalloc enc_coef");
  if (rc) return rc;
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
  rc = ensure_buf(&e->enc_coef, &e->enc_coef_cap, static_cast<size_t>(G) * k * rp + 64, "hipMalloc enc_coef");
  if (rc) return rc;
  hipStream_t st = static_cast<hipStream_t>(stream);
  PrepArgs p{};
  p.G = G; p.k = k; p.r = r; p.rp = rp; p.src_len = src_len; p.sid_base = sid_base;
  p.rid_base = rid_base; p.coef = static_cast<uint8_t*>(e->enc_coef); p.rep_size = rep_size;
  p.rep_len = rep_len;
  hipLaunchKernelGGL(encode_prep, dim3(G), dim3(256), 0, st, p);
  if ((rc = hip_check(hipGetLastError(), "encode_prep launch"))) return rc;
  const int D = pick_d(stride);
  MacArgs a{};
  a.G = G; a.k = k; a.rows = r; a.stride = stride;
  a.nrowchunks = (r + 31) / 32;
  a.ncolchunks = (stride + 256u * D - 1) / (256u * D);
  a.in0 = src; a.out = rep; a.coef = static_cast<const uint8_t*>(e->enc_coef); a.rp = rp;
  const uint64_t tasks = static_cast<uint64_t>(G) * a.nrowchunks * a.ncolchunks;
  const uint64_t blocks = (tasks + kWaves - 1) / kWaves;
  if (blocks > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "batch too large for one launch");
  hipLaunchKernelGGL(pick_kernel(false, D), dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, st, a);
  return hip_check(hipGetLastError(), "encode_mac launch");
}

int ntc_gf256_decode_plan(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                          uint16_t* src_len, const uint8_t* src_mask, const uint16_t* rep_size,
                          const uint8_t* rep_mask, const uint32_t* sid_base,
                          const uint32_t* rid_base, ntc_gf256_decode_status* status, void* stream)
{
  if (!e || !src_len || !src_mask || !rep_size || !rep_mask || !status)
    return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0) return fail(NTC_GPU_EINVAL, "G and k must be > 0");
  if (r > static_cast<uint32_t>(kMaxPlanRows)) return fail(NTC_GPU_EUNSUPPORTED, "r > 64 not supported by decode");
  if (k > 65535) return fail(NTC_GPU_EUNSUPPORTED, "k > 65535");
  const uint32_t rp = tile_rp(r);
  (void)hipSetDevice(e->device);
  int rc = ensure_plan(e, G, k, rp);
  if (rc) return rc;
  PlanArgs p{};
  p.G = G; p.k = k; p.r = r; p.src_len = src_len; p.src_mask = src_mask; p.rep_size = rep_size;
  p.rep_mask = rep_mask; p.sid_base = sid_base; p.rid_base = rid_base; p.status = status;
  p.plan_m = e->plan_m; p.plan_in = e->plan_in; p.plan_out = e->plan_out;
  p.plan_coef = e->plan_coef; p.rp = rp;
  hipLaunchKernelGGL(decode_plan, dim3(G), dim3(64), 0, static_cast<hipStream_t>(stream), p);
  e->last_G = G; e->last_k = k; e->last_r = r; e->last_rp = rp;
  return hip_check(hipGetLastError(), "decode_plan launch");
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
  const int D = pick_d(stride);
  MacArgs a{};
  a.G = G; a.k = k; a.rows = r; a.stride = stride;
  a.nrowchunks = (r + 31) / 32;
  a.ncolchunks = (stride + 256u * D - 1) / (256u * D);
  a.in0 = src; a.in1 = rep; a.out = src;
  a.rows_per_gen = e->plan_m; a.in_idx = e->plan_in; a.out_idx = e->plan_out;
  a.coef = e->plan_coef; a.rp = e->last_rp;
  const uint64_t tasks = static_cast<uint64_t>(G) * a.nrowchunks * a.ncolchunks;
  const uint64_t blocks = (tasks + kWaves - 1) / kWaves;
  if (blocks > 0x7FFFFFFFull) return fail(NTC_GPU_EUNSUPPORTED, "batch too large for one launch");
  hipLaunchKernelGGL(pick_kernel(true, D), dim3(static_cast<uint32_t>(blocks)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), a);
  return hip_check(hipGetLastError(), "decode_mac launch");
}

int ntc_gf256_decode_batch(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                           uint32_t stride, uint8_t* src, uint16_t* src_len,
                           const uint8_t* src_mask, const uint8_t* rep, const uint16_t* rep_size,
                           const uint8_t* rep_mask, const uint32_t* sid_base,
                           const uint32_t* rid_base, ntc_gf256_decode_status* status, void* stream)
{
  int rc = check_shape(G, k, r, stride);
  if (rc) return rc;
  rc = ntc_gf256_decode_plan(e, G, k, r, src_len, src_mask, rep_size, rep_mask, sid_base,
                             rid_base, status, stream);
  if (rc) return rc;
  return ntc_gf256_decode_apply(e, G, k, r, stride, src, rep, stream);
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
