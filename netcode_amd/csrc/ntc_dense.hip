// ntc_dense.hip -- dense GF(2^8) codes on MI355X (gfx950): batched device Gauss-Jordan + combine.
//
// BASELINE config 5 / SURVEY §8(f)3: k = 1024 sources, every one lost, k repairs each covering all
// k with a *non-reference* dense coefficient matrix (the reference's w = 8 schedule makes every such
// matrix singular: coefficient() has period 255, galois_field.hh:143-158).  Decoding is then
// "invert M, apply M^-1": the work of detail::invert (invert_matrix.cc:9-128) followed by the
// region MAC loop of attempt_full_decoding (detail/decoder.cc:503-534), at sizes the reference's
// m x m scalar path was never meant for.
//
// Inversion: blocked Gauss-Jordan on the augmented matrix X = [A | I] (np x 2np bytes per
// generation, np = n rounded up to the 32-column panel; A is embedded in the identity so padding
// never changes invertibility or the top-left block of the inverse).  Per panel of 32 columns:
//   dn_panel   one workgroup per generation, one thread per row (np <= 1024 threads): 32 pivot
//              steps over a 9-dword live window of the row (the panel columns still to eliminate
//              + the tracker columns already assigned), one barrier per step.  The tracker W
//              records the panel's row operations: afterwards
//                  row_i' = keep_i * row_i  XOR  sum_t W[t][i] * row_{piv_t}
//              with keep_i = 0 for the 32 rows chosen as pivots in this panel.
//   dn_update  applies that to the columns right of the panel (and the identity half) as a
//              GF(2^8) multiply-accumulate, X -> Y (ping-pong: pivot rows are read by every row).
// The default panel kernel is dn_panel_ra (run-ahead owner wave, no barrier per step); it leaves
// the trackers of non-pivot rows to dn_update, which derives them as W_i = X_i[panel] * T.
// Pivoting takes the lowest-index eligible row with a non-zero entry; the inverse is unique, so
// the result is the reference's M^-1 whatever the pivot order, and singularity is a rank property.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <string>

#include "engine.hh"
#include "gf256_field.hh"
#include "netcode/gpu.h"

namespace ntcgpu {
namespace dense {

__constant__ __attribute__((aligned(16))) PermTables dn_perm = make_perm_tables();
__constant__ __attribute__((aligned(16))) PermTables dn_pinv = make_inv_perm_tables();

constexpr uint32_t kPanel = 32;       // pivot columns per panel
constexpr uint32_t kMaxN = 1024;      // one thread per row in dn_panel
constexpr int kUpdRows = 4;           // rows per wave in dn_update
constexpr uint32_t kUpdSpan = 256;    // columns per wave in dn_update (64 lanes x 4 bytes)

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x16 __attribute__((ext_vector_type(16)));

// c*x for the four bytes of x; t = the 5 table dwords of c (PermTables layout, 3/3/2-bit split).
__device__ __forceinline__ uint32_t mul4(uint32_t t0, uint32_t t1, uint32_t t2, uint32_t t3,
                                         uint32_t t4, uint32_t x)
{
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(t1, t0, x & 0x07070707u),
                                     __builtin_amdgcn_perm(t3, t2, (x >> 3) & 0x07070707u),
                                     __builtin_amdgcn_perm(t4, t4, (x >> 6) & 0x03030303u), 0x96);
}

// A v_perm table set in LDS, split by dword so that per-lane gathers spread over the banks: the
// first four dwords of c's table at a 16-byte pitch (a ds_read_b128 of 16 lanes touches bank
// group c mod 16), the fifth at a 4-byte pitch (a ds_read_b32 of 32 lanes: bank c mod 32).  The
// PermTables layout (8 dwords per c) put every b128 gather on c mod 8 and every fifth-dword
// gather on c mod 4, 2-3x the LDS cycles of this one for random c.
struct LdsTab {
  u32x4 a[256];
  uint32_t b[256];
};

__device__ __forceinline__ void stage_tab(LdsTab& t, const PermTables& src, uint32_t tid, uint32_t n)
{
  for (uint32_t c = tid; c < 256; c += n) {
    u32x4 v;
    v[0] = src.w[c][0]; v[1] = src.w[c][1]; v[2] = src.w[c][2]; v[3] = src.w[c][3];
    t.a[c] = v;
    t.b[c] = src.w[c][4];
  }
}

__device__ __forceinline__ uint32_t lds_addr(const void* p)
{
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(
      reinterpret_cast<const __attribute__((address_space(3))) uint8_t*>(reinterpret_cast<uintptr_t>(p))));
}

template <typename T>
__device__ __forceinline__ T const_load(const void* p)
{
  return *reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p));
}

#ifdef NTC_DENSE_CLOCK
// Timeline of the lookahead launches (experiment builds only): per launch (index = the panel it
// factors), the panel block's stamps and the update blocks' first start / last end.
__device__ unsigned long long g_dn_clk[64 * 8];
#define DN_CLK(idx, slot)                                                    \
  do {                                                                       \
    if (threadIdx.x == 0) g_dn_clk[(idx) * 8 + (slot)] = wall_clock64();     \
  } while (0)
extern "C" int ntc_dbg_dense_clock(unsigned long long* out, uint32_t n, int reset)
{
  if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dn_clk), n * 8) != hipSuccess) return -1;
  if (reset) {
    static unsigned long long init[64 * 8];
    for (int i = 0; i < 64 * 8; ++i) init[i] = (i % 8 == 6) ? ~0ull : 0ull;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_dn_clk), init, sizeof(init)) != hipSuccess) return -1;
  }
  return 0;
}
#else
#define DN_CLK(idx, slot) do { } while (0)
#endif

// X[g] = [A | I]: A = mat[g] (n x n) inside an np x np identity.  Row flags: eligible = 1.
__global__ __launch_bounds__(256) void dn_init(const uint8_t* __restrict__ mat, uint32_t n,
                                               uint32_t np, uint8_t* __restrict__ X,
                                               uint8_t* __restrict__ flag, uint8_t* __restrict__ ok)
{
  const uint32_t i = blockIdx.x, g = blockIdx.y, P = 2 * np;
  uint8_t* row = X + (static_cast<size_t>(g) * np + i) * P;
  const uint8_t* mrow = mat + (static_cast<size_t>(g) * n + i) * n;
  for (uint32_t c = threadIdx.x; c < P; c += blockDim.x) {
    uint8_t v;
    if (c < np) v = (i < n && c < n) ? mrow[c] : static_cast<uint8_t>(i == c);
    else v = static_cast<uint8_t>(c - np == i);
    row[c] = v;
  }
  if (threadIdx.x == 0) {
    flag[static_cast<size_t>(g) * np + i] = 1;
    if (i == 0) ok[g] = 1;
  }
}

struct PanelArgs {
  uint32_t np, c0;
  const uint8_t* X;
  uint8_t* W;          // [G][np][32] tracker: row i's coefficients of the 32 pivot rows
  uint32_t* piv;       // [G][np] pivot row of column c
  uint8_t* flag;       // [G][np] 1 = not yet a pivot row (eligible)
  uint8_t* keep;       // [G][np] 0 = chosen as a pivot in this panel
  uint8_t* ok;         // [G] 0 once singular
};

// v_perm selector forms of a multiplicand dword x (a record word, a T word, a pivot-row word)
__device__ __forceinline__ u32x4 sel4(uint32_t x)
{
  u32x4 o;
  o[0] = x;
  o[1] = x & 0x07070707u;
  o[2] = (x >> 3) & 0x07070707u;
  o[3] = (x >> 6) & 0x03030303u;
  return o;
}

// c * x, c given by its table (tf, tf4; per lane), x by its selector forms (sel4)
__device__ __forceinline__ uint32_t mul_sel(const u32x4 tf, uint32_t tf4, const u32x4 c4)
{
  return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_perm(tf[1], tf[0], c4[1]),
                                     __builtin_amdgcn_perm(tf[3], tf[2], c4[2]),
                                     __builtin_amdgcn_perm(tf4, tf4, c4[3]), 0x96);
}

struct PanelSmem {
  LdsTab perm_t;                           // tables of c
  LdsTab pinv_t;                           // tables of 1/c
  u32x4 rec[kPanel][9];                    // step records
  // lookahead (dn_fused): the previous panel's T = B^-1 and its pivot rows' words in this
  // panel's columns, with their v_perm selectors; partial products of the cooperative pass
  u32x4 tsel[kPanel][8];
  u32x4 psel[kPanel][8];
  uint32_t stopv[2];                       // owner's stop step per phase
  uint32_t cm[2];                          // election masks per phase
  uint32_t ne[16];                         // wave has eligible rows
};

// Panel factorisation with a run-ahead owner wave: pivot order does not change the inverse, so
// the owner -- one wave that has a candidate -- eliminates the panel's columns on its own 64 rows
// for as many steps as it keeps finding candidates, writing one record per step (the normalised
// window with its v_perm selectors) and never waiting on the other waves.  One barrier later the
// other 15 waves apply every record in step order to their rows.  Only when the owner runs out of
// candidates at some column is there an election: every wave reports whether it has one, the
// lowest such wave becomes the next owner (none: singular).  A random dense matrix needs about one
// phase per panel, i.e. two barriers per 32 pivots instead of 32.
//
// LOOKAHEAD (dn_fused): the panel runs in the same launch as the previous panel's update, so its
// rows' panel columns are not in memory yet.  The block derives them for the owner wave's 64 rows
// from the pre-update matrix -- W_i = X_i[prev panel] * T, then X_i[panel] ^= sum_t W_i[t] *
// X[piv_t][panel], the update's own arithmetic, split over all waves -- and the other waves derive
// their own rows only if the owner does not finish the panel alone (an election).
// LOOKAHEAD: part = dynamic LDS of 2 x 8 x 64 dwords (the derivation's two ds_xor regions)
template <bool LOOKAHEAD>
__device__ __forceinline__ void panel_run(const PanelArgs& a, PanelSmem& sm, uint32_t g, uint32_t i,
                                          uint32_t nthreads, uint32_t* part = nullptr)
{
  const uint32_t lane = i & 63u, w = i >> 6, nw = nthreads >> 6;
  const uint32_t np = a.np, P = 2 * np;
  const bool row_ok = i < np;
  const size_t gi = static_cast<size_t>(g) * np + i;
  bool elig = row_ok && a.flag[gi] != 0;
  const uint32_t cp = a.c0 - kPanel;                   // LOOKAHEAD: the previous panel's columns
  if (LOOKAHEAD && g == 0) DN_CLK(a.c0 / kPanel, 0);
  // LOOKAHEAD with >= 256 threads: two rounds of loads before the staging barrier -- (1) the
  // previous pivots, all row flags (16 per lane) and the tables; (2) the pivot rows' T and panel
  // words, and the owner rows' words the derivation needs (the owner = the wave of the lowest
  // eligible row, known from the flags), so the derivation starts with its operands in registers
  uint32_t owner_e = 0, xq0 = 0, xq1 = 0;
  u32x4 own0 = {0, 0, 0, 0}, own1 = {0, 0, 0, 0};
  const bool early = LOOKAHEAD && nthreads >= kPanel * 8;
  if (early) {
    const bool st = i < kPanel * 8;
    const uint32_t s_ = i >> 3, d_ = i & 7u;
    // a generation that went singular stopped writing pivots (and one that was singular from the
    // start never wrote any): its entries are stale or uninitialised, so clamp them into the
    // generation's rows -- the words loaded for a dead generation are never used (!live below)
    const uint32_t pr = st ? min(a.piv[static_cast<size_t>(g) * np + cp + s_], np - 1u) : 0u;
    const uint32_t r0 = lane * 16u;
    u32x4 fl = {0, 0, 0, 0};
    if (r0 < np) fl = *reinterpret_cast<const u32x4*>(a.flag + static_cast<size_t>(g) * np + r0);
    stage_tab(sm.perm_t, dn_perm, i, nthreads);
    stage_tab(sm.pinv_t, dn_pinv, i, nthreads);
    uint32_t fidx = ~0u;
#pragma unroll
    for (int d = 3; d >= 0; --d)
      if (fl[d] != 0) fidx = 4u * d + (__builtin_ctz(fl[d]) >> 3);
    const uint64_t fb = __ballot(fidx != ~0u);
    if (fb != 0) {
      const uint32_t fl_lane = __ffsll(static_cast<long long>(fb)) - 1;
      owner_e = (16u * fl_lane + __builtin_amdgcn_readlane(fidx, fl_lane)) >> 6;
    }
    owner_e = __builtin_amdgcn_readfirstlane(owner_e);
    const uint32_t orow = owner_e * 64u + lane;
    if (orow < np) {
      const uint8_t* xo = a.X + (static_cast<size_t>(g) * np + orow) * P;
      if (w < kPanel) xq0 = *reinterpret_cast<const uint32_t*>(xo + cp + (w & ~3u));
      if (w + nw < kPanel) xq1 = *reinterpret_cast<const uint32_t*>(xo + cp + ((w + nw) & ~3u));
      if (w == owner_e) {
        own0 = reinterpret_cast<const u32x4*>(xo + a.c0)[0];
        own1 = reinterpret_cast<const u32x4*>(xo + a.c0)[1];
      }
    }
    if (st) {
      const size_t prow = static_cast<size_t>(g) * np + pr;
      const uint32_t wv = *reinterpret_cast<const uint32_t*>(a.W + prow * kPanel + 4 * d_);
      const uint32_t xv = *reinterpret_cast<const uint32_t*>(a.X + prow * P + a.c0 + 4 * d_);
      sm.tsel[s_][d_] = sel4(wv);
      sm.psel[s_][d_] = sel4(xv);
    }
  } else {
    stage_tab(sm.perm_t, dn_perm, i, nthreads);
    stage_tab(sm.pinv_t, dn_pinv, i, nthreads);
    if (LOOKAHEAD) {
      const uint32_t* pivp = a.piv + static_cast<size_t>(g) * np + cp;
      for (uint32_t e = i; e < kPanel * 8; e += nthreads) {
        const uint32_t s = e >> 3, d = e & 7;
        const size_t prow = static_cast<size_t>(g) * np + min(pivp[s], np - 1u);   // as above
        sm.tsel[s][d] = sel4(*reinterpret_cast<const uint32_t*>(a.W + prow * kPanel + 4 * d));
        sm.psel[s][d] = sel4(*reinterpret_cast<const uint32_t*>(a.X + prow * P + a.c0 + 4 * d));
      }
    }
  }
  if (LOOKAHEAD)                                       // the derivation's two ds_xor regions
    for (uint32_t e = i; e < 2u * 8u * 64u; e += nthreads) part[e] = 0;
  if (i < 2) sm.cm[i] = 0;
  {
    const uint64_t e0 = __ballot(elig);
    if (lane == 0) sm.ne[w] = e0 != 0 ? 1u : 0u;
  }
  const bool live = a.ok[g] != 0;
  __syncthreads();
  if (LOOKAHEAD && g == 0) DN_CLK(a.c0 / kPanel, 1);
  if (!live) return;                                   // uniform: a singular generation stops
  uint32_t owner = owner_e;
  if (!early)
    for (uint32_t q = nw; q-- > 0;) owner = sm.ne[q] ? q : owner;
  owner = __builtin_amdgcn_readfirstlane(owner);

  uint32_t v[16];
#pragma unroll
  for (int d = 0; d < 16; ++d) v[d] = 0;
  bool have = !LOOKAHEAD;                              // this wave's rows hold the panel columns
  if (!LOOKAHEAD) {
    if (row_ok) {
      const u32x4* src = reinterpret_cast<const u32x4*>(a.X + gi * P + a.c0);
      const u32x4 q0 = src[0], q1 = src[1];
      v[0] = q0[0]; v[1] = q0[1]; v[2] = q0[2]; v[3] = q0[3];
      v[4] = q1[0]; v[5] = q1[1]; v[6] = q1[2]; v[7] = q1[3];
    }
  } else {
    // the owner's 64 rows, all waves: wave w takes the terms s = w, w + nw, ... of W_i (phase 1)
    // and then of the panel columns (phase 2), all 8 words each -- every table is gathered once
    // per lane -- and XOR-accumulates its partial words into LDS (ds_xor): region 1 = W_i,
    // region 2 = the owner rows' panel words, zeroed before the staging barrier
    const uint32_t orow = owner * 64u + lane;
    const bool orow_ok = orow < np;
    const size_t go = static_cast<size_t>(g) * np + (orow_ok ? orow : 0u);
    if (!early && w == owner && orow_ok) {
      const u32x4* src = reinterpret_cast<const u32x4*>(a.X + go * P + a.c0);
      own0 = src[0];
      own1 = src[1];
    }
    auto xor_words = [&](uint32_t* region, const uint32_t (&acc)[8]) {
#pragma unroll
      for (int d = 0; d < 8; ++d)
        __hip_atomic_fetch_xor(&region[d * 64u + lane], acc[d], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    {
      uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t s = w; s < kPanel; s += nw) {
        const uint32_t xq = early && s == w ? xq0 : early && s == w + nw ? xq1
                          : orow_ok ? *reinterpret_cast<const uint32_t*>(a.X + go * P + cp + (s & ~3u)) : 0u;
        const uint32_t b = (xq >> (8 * (s & 3))) & 0xFFu;
        const u32x4 tf = sm.perm_t.a[b];
        const uint32_t tf4 = sm.perm_t.b[b];
#pragma unroll
        for (int d = 0; d < 8; ++d) acc[d] ^= mul_sel(tf, tf4, sm.tsel[s][d]);
      }
      xor_words(part, acc);
    }
    __syncthreads();
    {
      uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (uint32_t t = w; t < kPanel; t += nw) {
        const uint32_t b = (part[(t >> 2) * 64u + lane] >> (8 * (t & 3))) & 0xFFu;
        const u32x4 tf = sm.perm_t.a[b];
        const uint32_t tf4 = sm.perm_t.b[b];
#pragma unroll
        for (int d = 0; d < 8; ++d) acc[d] ^= mul_sel(tf, tf4, sm.psel[t][d]);
      }
      xor_words(part + 512u, acc);
    }
    __syncthreads();
    if (w == owner) {
      const uint32_t x8[8] = {own0[0], own0[1], own0[2], own0[3], own1[0], own1[1], own1[2], own1[3]};
#pragma unroll
      for (int d = 0; d < 8; ++d) v[d] = orow_ok ? x8[d] ^ part[512u + d * 64u + lane] : 0u;
      have = true;
    }
    if (g == 0) DN_CLK(a.c0 / kPanel, 2);
  }
  // LOOKAHEAD, a wave that is needed after all: its rows' panel columns on its own
  auto materialise = [&]() {
    if (have) return;
    have = true;
    if (!row_ok) return;
    // (the rare path: kept small -- a loop over the words, not unrolled)
    uint32_t wi[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      const uint32_t xq = *reinterpret_cast<const uint32_t*>(a.X + gi * P + cp + 4 * q);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = (xq >> (8 * k)) & 0xFFu;
        const u32x4 tf = sm.perm_t.a[b];
        const uint32_t tf4 = sm.perm_t.b[b];
#pragma unroll
        for (int d = 0; d < 8; ++d) wi[d] ^= mul_sel(tf, tf4, sm.tsel[4 * q + k][d]);
      }
    }
    const u32x4* xc = reinterpret_cast<const u32x4*>(a.X + gi * P + a.c0);
    const u32x4 c0v = xc[0], c1v = xc[1];
    v[0] = c0v[0]; v[1] = c0v[1]; v[2] = c0v[2]; v[3] = c0v[3];
    v[4] = c1v[0]; v[5] = c1v[1]; v[6] = c1v[2]; v[7] = c1v[3];
#pragma unroll 1
    for (int q = 0; q < 8; ++q) {
      uint32_t wq = 0;
#pragma unroll
      for (int qq = 0; qq < 8; ++qq) wq = qq == q ? wi[qq] : wq;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = (wq >> (8 * k)) & 0xFFu;
        const u32x4 tf = sm.perm_t.a[b];
        const uint32_t tf4 = sm.perm_t.b[b];
#pragma unroll
        for (int d = 0; d < 8; ++d) v[d] ^= mul_sel(tf, tf4, sm.psel[4 * q + k][d]);
      }
    }
  };
  bool chosen = false;
  bool singular = false;

  // row -= f * record s (window of step s)
  auto apply = [&](int s) {
    const int q = s >> 2, sh = 8 * (s & 3);
    auto wd = [q](int e) { return e < 8 - q ? q + e : 8 + (e - (8 - q)); };
    const uint32_t f = (v[q] >> sh) & 0xFFu;
    if (f != 0) {
      const u32x4 tf = sm.perm_t.a[f];
      const uint32_t tf4 = sm.perm_t.b[f];
#pragma unroll
      for (int e = 0; e < 9; ++e) v[wd(e)] ^= mul_sel(tf, tf4, sm.rec[s][e]);
    }
  };
  uint32_t t = 0;
  for (uint32_t phase = 0;; ++phase) {
    const uint32_t par = phase & 1u;
    if (w == owner) {                                    // wave-uniform: run ahead from step t
      // One step: ballot of the rows with a non-zero in column s, the pivot row's nine window
      // words into lanes 0-8 (v_readlane -> v_writelane), normalised there by the pivot's 1/f
      // table (v_readlane'd from its lane) and written to LDS as the step's record with its v_perm
      // selectors, then every row's update from the record (the pivot row takes the record by a
      // select).  Software-pipelined: step s + 1's table gathers are issued right after the word
      // of column s + 1 is updated and land under the rest of step s's update.  Those gathers and
      // the record reads are inline asm, so the compiler can neither sink the gathers below the
      // next ballot nor make a record read wait on them (LDS returns in order: every record read
      // is issued before the gathers).  Measured slower (round 4): the record as v_readlane'd
      // uniform words with scalar selectors instead of the LDS round trip, one branch-free block
      // per phase, and the same pipelining with compiler-placed loads.
      uint32_t stop = kPanel;
      const uint32_t pa0 = lds_addr(&sm.perm_t.a[0]), pb0 = lds_addr(&sm.perm_t.b[0]);
      const uint32_t ia0 = lds_addr(&sm.pinv_t.a[0]), ib0 = lds_addr(&sm.pinv_t.b[0]);
      const uint32_t rec0 = lds_addr(&sm.rec[0][0]);
      u32x4 tfn, tln;
      uint32_t tf4n, tl4n;
      auto gather = [&](uint32_t fv) {
        asm volatile("ds_read_b128 %0, %1" : "=v"(tfn) : "v"(pa0 + 16u * fv));
        asm volatile("ds_read_b32 %0, %1" : "=v"(tf4n) : "v"(pb0 + 4u * fv));
        asm volatile("ds_read_b128 %0, %1" : "=v"(tln) : "v"(ia0 + 16u * fv));
        asm volatile("ds_read_b32 %0, %1" : "=v"(tl4n) : "v"(ib0 + 4u * fv));
      };
      uint32_t fn = 0;
#pragma unroll
      for (int s = 0; s < static_cast<int>(kPanel); ++s)
        if (s == static_cast<int>(t)) fn = (v[s >> 2] >> (8 * (s & 3))) & 0xFFu;
      gather(fn);
      uint64_t elig_m = __ballot(elig);                 // the eligible rows as a wave mask
      uint32_t pv = 0;                                   // lane s: the pivot row of step s
#pragma unroll
      for (int s = 0; s < static_cast<int>(kPanel); ++s) {
        if (s < static_cast<int>(t)) continue;
        const int q = s >> 2, sh = 8 * (s & 3);
        auto wd = [q](int e) { return e < 8 - q ? q + e : 8 + (e - (8 - q)); };
        const uint32_t f = fn;
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(tfn), "+v"(tf4n), "+v"(tln), "+v"(tl4n));
        const u32x4 tf = tfn, tl = tln;
        const uint32_t tf4 = tf4n, tl4 = tl4n;
        const uint64_t b = __ballot(f != 0) & elig_m;
        if (b == 0) { stop = s; break; }
        const uint32_t first = __ffsll(static_cast<long long>(b)) - 1;
        uint32_t x = 0;
#pragma unroll
        for (int e = 0; e < 9; ++e) {
          uint32_t val = __builtin_amdgcn_readlane(v[wd(e)], first);
          if (wd(e) == 8 + q) val ^= 1u << sh;
          asm("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(val), "i"(e));
        }
        u32x4 ti;
        ti[0] = __builtin_amdgcn_readlane(tl[0], first);
        ti[1] = __builtin_amdgcn_readlane(tl[1], first);
        ti[2] = __builtin_amdgcn_readlane(tl[2], first);
        ti[3] = __builtin_amdgcn_readlane(tl[3], first);
        const uint32_t ti4 = __builtin_amdgcn_readlane(tl4, first);
        if (lane < 9) sm.rec[s][lane] = sel4(mul4(ti[0], ti[1], ti[2], ti[3], ti4, x));
        __builtin_amdgcn_wave_barrier();
        asm("v_writelane_b32 %0, %1, %2" : "+v"(pv) : "s"(__builtin_amdgcn_readfirstlane(w * 64u + first)), "i"(s));
        const bool me = lane == first;
        const int en = (s + 1 < static_cast<int>(kPanel)) ? (((s + 1) >> 2) - q) : 0;
        // the record's nine entries read by inline asm too, the next column's first, so that
        // every read is older than the next step's gathers (LDS returns in order: waiting for the
        // record never waits for the gathers).  The lgkmcnt values below are hand-counted: they
        // hold only while the compiler issues no other LGKM operation in this window and does not
        // copy an asm output register before its wait ("+v" on the wait is the only tie).
        // Verified on ROCm 7.2 (AMD clang 22.0.0git, roc-7.2.0 26014) by disassembly; a compiler
        // that breaks either assumption produces wrong pivot records, which the dense parity
        // suite (tests/test_gpu_dense.py, inverses against the oracle) reports.
        u32x4 c[9];
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(c[en]) : "v"(rec0), "i"((s * 9 + en) * 16));
#pragma unroll
        for (int e = 0; e < 9; ++e)
          if (e != en) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(c[e]) : "v"(rec0), "i"((s * 9 + e) * 16));
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(c[en]));
        auto upd = [&](int e) {
          const u32x4 c4 = c[e];
          const uint32_t u = __builtin_amdgcn_bitop3_b32(v[wd(e)], __builtin_amdgcn_perm(tf[1], tf[0], c4[1]),
                                                         __builtin_amdgcn_perm(tf[3], tf[2], c4[2]), 0x96) ^
                             __builtin_amdgcn_perm(tf4, tf4, c4[3]);
          v[wd(e)] = me ? c4[0] : u;
        };
        upd(en);
        if (s + 1 < static_cast<int>(kPanel)) {
          fn = (v[(s + 1) >> 2] >> (8 * ((s + 1) & 3))) & 0xFFu;
          gather(fn);
          asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]),
                       "+v"(c[5]), "+v"(c[6]), "+v"(c[7]), "+v"(c[8]));
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(c[0]), "+v"(c[1]), "+v"(c[2]), "+v"(c[3]), "+v"(c[4]),
                       "+v"(c[5]), "+v"(c[6]), "+v"(c[7]), "+v"(c[8]));
        }
#pragma unroll
        for (int e = 0; e < 9; ++e)
          if (e != en) upd(e);
        elig_m &= ~(1ull << first);
        if (me) { chosen = true; elig = false; }
      }
      // this phase's pivots, one store
      if (lane >= t && lane < stop) a.piv[static_cast<size_t>(g) * np + a.c0 + lane] = pv;
      if (lane == 0) sm.stopv[par] = stop;
    }
    __syncthreads();
    if (LOOKAHEAD && g == 0 && phase == 0) DN_CLK(a.c0 / kPanel, 3);
    const uint32_t stop = __builtin_amdgcn_readfirstlane(sm.stopv[par]);
    // the other waves need the records only to elect (phase incomplete) or to finish rows they
    // gave as pivots in an earlier phase; the trackers of non-pivot rows come from dn_update
    const bool need = stop < kPanel || __ballot(chosen) != 0;
    if (w != owner && need) {
      materialise();
#pragma unroll
      for (int s = 0; s < static_cast<int>(kPanel); ++s)
        if (s >= static_cast<int>(t) && s < static_cast<int>(stop)) apply(s);
    }
    t = stop;
    if (t >= kPanel) break;
    // election at column t: the lowest wave with a candidate owns the next phase
    uint32_t f = 0;
#pragma unroll
    for (int s = 0; s < static_cast<int>(kPanel); ++s)
      if (s == static_cast<int>(t)) f = (v[s >> 2] >> (8 * (s & 3))) & 0xFFu;
    const uint64_t b = __ballot(elig && f != 0);
    if (b != 0 && lane == 0) atomicOr(&sm.cm[par], 1u << w);
    __syncthreads();
    const uint32_t m = __builtin_amdgcn_readfirstlane(sm.cm[par]);
    if (i == 0) sm.cm[par ^ 1u] = 0;                     // next read after two more barriers
    if (m == 0) { singular = true; break; }              // uniform
    owner = __ffs(m) - 1;
  }
  if (singular) {
    if (i == 0) a.ok[g] = 0;
    return;
  }
  if (row_ok) {
    a.flag[gi] = elig ? 1 : 0;
    a.keep[gi] = chosen ? 0 : 1;
  }
  if (LOOKAHEAD && g == 0) DN_CLK(a.c0 / kPanel, 4);
  if (chosen) {                                        // T: the pivot rows' trackers only
    u32x4* wg = reinterpret_cast<u32x4*>(a.W + gi * kPanel);
    u32x4 o0, o1;
    o0[0] = v[8]; o0[1] = v[9]; o0[2] = v[10]; o0[3] = v[11];
    o1[0] = v[12]; o1[1] = v[13]; o1[2] = v[14]; o1[3] = v[15];
    wg[0] = o0;
    wg[1] = o1;
  }
}

__global__ __launch_bounds__(1024) void dn_panel_ra(PanelArgs a)
{
  __shared__ __attribute__((aligned(16))) PanelSmem sm;
  panel_run<false>(a, sm, blockIdx.x, threadIdx.x, blockDim.x);
}

struct UpdArgs {
  uint32_t G, np, c0, cs;      // cs: first column to produce
  uint32_t ntiles, nspans;
  const uint8_t* X;
  uint8_t* Y;
  const uint8_t* W;
  const uint32_t* piv;
  const uint8_t* keep;
  const uint8_t* ok;
};

// One update task (a wave) per (generation, 4-row tile, 256-column span of [cs, 2np)), 4 bytes
// per lane:  Y[i][c] = keep_i * X[i][c]  XOR  sum_t W[t][i] * X[piv_t][c].
// Pivot-row slices stream in groups of 8 with the next group's loads in flight; v_perm tables come
// from an LDS copy (uniform addresses: broadcast reads).  Narrow spans keep >= 2 waves per SIMD
// at n = 1024 (G = 1), which this latency-bound kernel needs.
struct UpdSmem {
  LdsTab perm_t;
  uint32_t tT[16][kPanel * 8];             // per wave: T by step
};

__device__ __forceinline__ void update_task(const UpdArgs& a, uint32_t task, uint32_t lane, uint32_t* tT,
                                            const LdsTab& perm_t)
{
  task = __builtin_amdgcn_readfirstlane(task);
  const uint32_t span = task % a.nspans;
  task /= a.nspans;
  const uint32_t tile = task % a.ntiles;
  const uint32_t g = task / a.ntiles;
  if (g >= a.G) return;
  if (__builtin_amdgcn_readfirstlane(a.ok[g]) == 0) return;
  const uint32_t np = a.np, P = 2 * np;
  const uint32_t col = a.cs + span * kUpdSpan + lane * 4u;
  const bool active = col < P;
  const uint32_t cx = active ? col : a.cs;
  const uint8_t* Xg = a.X + static_cast<size_t>(g) * np * P + cx;
  uint8_t* Yg = a.Y + static_cast<size_t>(g) * np * P;
  const uint32_t i0 = tile * kUpdRows;
  const uint32_t* piv = a.piv + static_cast<size_t>(g) * np + a.c0;
  const uint32_t kw = const_load<uint32_t>(a.keep + static_cast<size_t>(g) * np + i0);
  // The tile's 4 x 32 tracker bytes, byte t of row j = word 8j + t/4, moved to SGPRs.  A pivot
  // row's tracker is the panel's (its row of T = B^-1, B = the pivot rows' panel columns); any
  // other row's is derived here, not by the panel: its panel columns vanish, so
  // W_i = X_i[c0 .. c0 + 32) * T -- 32 products per tracker dword, lane 8j + d holding dword d of
  // row j, T staged in this wave's LDS slice.
  uint32_t wv[4 * kUpdRows * 2];
  {
    {
      const uint32_t s = lane >> 1, h = lane & 1u;
      const u32x4 q = *reinterpret_cast<const u32x4*>(
          a.W + (static_cast<size_t>(g) * np + piv[s]) * kPanel + 16u * h);
      *reinterpret_cast<u32x4*>(&tT[8 * s + 4 * h]) = q;
    }
    const uint32_t j = (lane >> 3) & 3u, d = lane & 7u;
    const u32x4* xr = reinterpret_cast<const u32x4*>(a.X + (static_cast<size_t>(g) * np + i0 + j) * P + a.c0);
    const u32x4 x0 = xr[0], x1 = xr[1];
    const uint32_t xw[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
    __builtin_amdgcn_wave_barrier();
    uint32_t acc_w = 0;
#pragma unroll
    for (int s = 0; s < static_cast<int>(kPanel); ++s) {
      const uint32_t c = (xw[s >> 2] >> (8 * (s & 3))) & 0xFFu;
      const u32x4 tab = perm_t.a[c];
      const uint32_t t4 = perm_t.b[c];
      acc_w ^= mul4(tab[0], tab[1], tab[2], tab[3], t4, tT[8 * s + d]);
    }
    if (((kw >> (8 * j)) & 0xFFu) == 0)
      acc_w = *reinterpret_cast<const uint32_t*>(a.W + (static_cast<size_t>(g) * np + i0 + j) * kPanel + 4u * d);
#pragma unroll
    for (int q = 0; q < 4 * kUpdRows * 2; ++q) wv[q] = __builtin_amdgcn_readlane(acc_w, q);
  }

  uint32_t acc[kUpdRows];
#pragma unroll
  for (int j = 0; j < kUpdRows; ++j)
    acc[j] = ((kw >> (8 * j)) & 0xFFu) ? *reinterpret_cast<const uint32_t*>(Xg + static_cast<size_t>(i0 + j) * P) : 0u;
  constexpr uint32_t kGrp = 8;
  uint32_t xc[kGrp];
  {
    const u32x8 pg = const_load<u32x8>(piv);
#pragma unroll
    for (uint32_t u = 0; u < kGrp; ++u) xc[u] = *reinterpret_cast<const uint32_t*>(Xg + static_cast<size_t>(pg[u]) * P);
  }
#pragma unroll
  for (uint32_t grp = 0; grp < kPanel / kGrp; ++grp) {
    uint32_t xn[kGrp];
    if (grp + 1 < kPanel / kGrp) {
      const u32x8 pg = const_load<u32x8>(piv + kGrp * (grp + 1));
#pragma unroll
      for (uint32_t u = 0; u < kGrp; ++u) xn[u] = *reinterpret_cast<const uint32_t*>(Xg + static_cast<size_t>(pg[u]) * P);
    }
#pragma unroll
    for (uint32_t u = 0; u < kGrp; ++u) {
      const uint32_t t = kGrp * grp + u;
      const uint32_t sa = xc[u] & 0x07070707u, sb = (xc[u] >> 3) & 0x07070707u, se = (xc[u] >> 6) & 0x03030303u;
#pragma unroll
      for (int j = 0; j < kUpdRows; ++j) {
        const uint32_t wi = 8u * j + (t >> 2);
        const uint32_t c = (wv[wi] >> (8 * (t & 3))) & 0xFFu;   // 0: zero table
        const u32x4 tab = perm_t.a[c];
        const uint32_t t4 = perm_t.b[c];
        acc[j] = __builtin_amdgcn_bitop3_b32(acc[j], __builtin_amdgcn_perm(tab[1], tab[0], sa),
                                             __builtin_amdgcn_perm(tab[3], tab[2], sb), 0x96) ^
                 __builtin_amdgcn_perm(t4, t4, se);
      }
    }
    if (grp + 1 < kPanel / kGrp) {
#pragma unroll
      for (uint32_t u = 0; u < kGrp; ++u) xc[u] = xn[u];
    }
  }
  if (!active) return;
#pragma unroll
  for (int j = 0; j < kUpdRows; ++j) *reinterpret_cast<uint32_t*>(Yg + static_cast<size_t>(i0 + j) * P + col) = acc[j];
}

__global__ __launch_bounds__(256) void dn_update(UpdArgs a)        // one task per wave
{
  __shared__ __attribute__((aligned(16))) LdsTab perm_t;
  __shared__ __attribute__((aligned(16))) uint32_t tT_all[4][kPanel * 8];
  stage_tab(perm_t, dn_perm, threadIdx.x, 256);
  __syncthreads();
  update_task(a, blockIdx.x * 4u + (threadIdx.x >> 6), threadIdx.x & 63u, tT_all[threadIdx.x >> 6], perm_t);
}

struct FusedArgs {
  PanelArgs pa;                // panel p + 1 (LOOKAHEAD)
  UpdArgs ua;                  // update of panel p
  uint32_t nA;                 // blocks [0, nA): one panel per generation; the rest: update tasks
  uint32_t tpb;                // update tasks (waves) per block
};

// Panel p + 1 beside the update of panel p, in one launch: the panel's owner chain runs while the
// other CUs apply panel p (they touch disjoint state: the update reads keep / W / piv of panel p
// and writes Y; the panel reads X, writes piv of its own columns, flags, the other keep buffer and
// the trackers of rows not chosen in panel p).
__global__ __launch_bounds__(1024) void dn_fused(FusedArgs f)
{
  __shared__ __attribute__((aligned(16))) union {
    PanelSmem p;
    UpdSmem u;
  } sm;
  if (blockIdx.x < f.nA) {
    extern __shared__ __attribute__((aligned(16))) uint32_t dn_part[];
    panel_run<true>(f.pa, sm.p, blockIdx.x, threadIdx.x, blockDim.x, dn_part);
    return;
  }
#ifdef NTC_DENSE_CLOCK
  if (threadIdx.x == 0) atomicMin(&g_dn_clk[(f.pa.c0 / kPanel) * 8 + 6], wall_clock64());
#endif
  stage_tab(sm.u.perm_t, dn_perm, threadIdx.x, blockDim.x);
  __syncthreads();
  const uint32_t w = threadIdx.x >> 6;
  if (w < f.tpb) update_task(f.ua, (blockIdx.x - f.nA) * f.tpb + w, threadIdx.x & 63u, sm.u.tT[w], sm.u.perm_t);
#ifdef NTC_DENSE_CLOCK
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&g_dn_clk[(f.pa.c0 / kPanel) * 8 + 7], wall_clock64());
#endif
}

// inv[g][t][0..n) = X[g][piv[t]][np .. np + n)  (zeros for a singular generation)
__global__ __launch_bounds__(256) void dn_gather_inv(uint32_t n, uint32_t np, const uint8_t* __restrict__ X,
                                                     const uint32_t* __restrict__ piv,
                                                     const uint8_t* __restrict__ ok, uint8_t* __restrict__ inv)
{
  const uint32_t t = blockIdx.x, g = blockIdx.y, P = 2 * np;
  const bool good = ok[g] != 0;
  const uint8_t* src = X + (static_cast<size_t>(g) * np + (good ? piv[static_cast<size_t>(g) * np + t] : 0)) * P + np;
  uint8_t* dst = inv + (static_cast<size_t>(g) * n + t) * n;
  for (uint32_t c = threadIdx.x; c < n; c += blockDim.x) dst[c] = good ? src[c] : 0;
}

// dst[g][c][r] = src[g][r][c] (src [G][R][C], dst [G][C][pitch], pitch >= R; entries r >= R of a
// dst row are zeroed).  64 x 64 tiles through LDS.
__global__ __launch_bounds__(256) void dn_transpose(uint32_t R, uint32_t C, uint32_t pitch,
                                                    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst)
{
  __shared__ uint8_t tile[64][65];
  const uint32_t g = blockIdx.z;
  const uint32_t r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const uint32_t tx = threadIdx.x & 63u, ty = threadIdx.x >> 6;
  const uint8_t* s = src + static_cast<size_t>(g) * R * C;
  for (uint32_t y = ty; y < 64; y += 4) {
    const uint32_t r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < R && c < C) ? s[static_cast<size_t>(r) * C + c] : 0;
  }
  __syncthreads();
  uint8_t* d = dst + static_cast<size_t>(g) * C * pitch;
  for (uint32_t y = ty; y < 64; y += 4) {
    const uint32_t c = c0 + y, r = r0 + tx;
    if (c < C && r < pitch) d[static_cast<size_t>(c) * pitch + r] = tile[tx][y];
  }
}

}  // namespace dense
}  // namespace ntcgpu

using namespace ntcgpu;
using namespace ntcgpu::dense;

namespace {

// NTC_DENSE_LOOKAHEAD=0: panel and update in separate launches (A/B experiments)
bool dense_lookahead()
{
  static const bool on = [] {
    const char* v = std::getenv("NTC_DENSE_LOOKAHEAD");
    return !v || std::atoi(v) != 0;
  }();
  return on;
}

// Blocked Gauss-Jordan of G n x n matrices; on return (stream order) the inverse rows sit in the
// engine's X buffer (rows permuted by piv) and ok[g] says whether generation g was invertible.
int dense_invert(ntc_gf256_engine* e, uint32_t G, uint32_t n, const uint8_t* mat, hipStream_t st,
                 const uint8_t** Xout, uint32_t* np_out)
{
  const uint32_t np = (n + kPanel - 1) / kPanel * kPanel;
  const size_t xb = static_cast<size_t>(G) * np * 2 * np;
  int rc;
  if ((rc = ensure_buf(e, &e->dn_x, &e->dn_x_cap, xb, "hipMalloc dense X"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_y, &e->dn_y_cap, xb, "hipMalloc dense Y"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_w, &e->dn_w_cap, static_cast<size_t>(G) * kPanel * np + 16, "hipMalloc dense W"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_piv, &e->dn_piv_cap, static_cast<size_t>(G) * np * 4 + 16, "hipMalloc dense piv"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_flag, &e->dn_flag_cap, static_cast<size_t>(G) * np * 3 + 16, "hipMalloc dense flags"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_ok, &e->dn_ok_cap, G + 16, "hipMalloc dense ok"))) return rc;
  uint8_t* X = static_cast<uint8_t*>(e->dn_x);
  uint8_t* Y = static_cast<uint8_t*>(e->dn_y);
  uint8_t* flag = static_cast<uint8_t*>(e->dn_flag);
  // keep flags by panel parity: with lookahead, panel p + 1 writes its own while p's update reads
  uint8_t* keep[2] = {flag + static_cast<size_t>(G) * np, flag + static_cast<size_t>(G) * np * 2};
  uint8_t* ok = static_cast<uint8_t*>(e->dn_ok);
  uint8_t* W = static_cast<uint8_t*>(e->dn_w);
  uint32_t* piv = static_cast<uint32_t*>(e->dn_piv);
  hipLaunchKernelGGL(dn_init, dim3(np, G), dim3(256), 0, st, mat, n, np, X, flag, ok);
  if ((rc = hip_check(hipGetLastError(), "dn_init launch"))) return rc;
  const uint32_t threads = (np + 63) / 64 * 64;
  const uint32_t npan = np / kPanel;
  auto upd_args = [&](uint32_t p) {
    UpdArgs ua{};
    const uint32_t c0 = p * kPanel;
    ua.G = G; ua.np = np; ua.c0 = c0;
    // the A half left of the next panel is never read again; the last panel only needs the I half
    ua.cs = c0 + kPanel < np ? c0 + kPanel : np;
    ua.ntiles = np / kUpdRows;
    ua.nspans = (2 * np - ua.cs + kUpdSpan - 1) / kUpdSpan;
    ua.X = X; ua.Y = Y; ua.W = W; ua.piv = piv; ua.keep = keep[p & 1]; ua.ok = ok;
    return ua;
  };
  auto panel_args = [&](uint32_t p) {
    return PanelArgs{np, p * kPanel, X, W, piv, flag, keep[p & 1], ok};
  };
  PanelArgs pa0 = panel_args(0);
  hipLaunchKernelGGL(dn_panel_ra, dim3(G), dim3(threads), 0, st, pa0);
  if ((rc = hip_check(hipGetLastError(), "dn_panel launch"))) return rc;
  for (uint32_t p = 0; p < npan; ++p) {
    const UpdArgs ua = upd_args(p);
    const uint64_t waves = static_cast<uint64_t>(G) * ua.ntiles * ua.nspans;
    if (p + 1 < npan && dense_lookahead()) {
      // update p and panel p + 1 in one launch; update tasks spread over the CUs the panels leave
      FusedArgs fa{};
      fa.pa = panel_args(p + 1);
      fa.ua = ua;
      fa.nA = G;
      const uint32_t nw = threads / 64;
      const uint64_t spread = G < 240 ? 240 - G : 16;
      fa.tpb = static_cast<uint32_t>(std::min<uint64_t>(nw, std::max<uint64_t>(1, (waves + spread - 1) / spread)));
      const uint64_t nb = (waves + fa.tpb - 1) / fa.tpb;
      const size_t part_bytes = 2 * 8 * 64 * 4;        // the derivation's two ds_xor regions
      static const bool attr = hipFuncSetAttribute(reinterpret_cast<const void*>(dn_fused),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   static_cast<int>(17 * 8 * 64 * 4)) == hipSuccess;
      (void)attr;
      hipLaunchKernelGGL(dn_fused, dim3(static_cast<uint32_t>(G + nb)), dim3(threads), part_bytes, st, fa);
      if ((rc = hip_check(hipGetLastError(), "dn_fused launch"))) return rc;
    } else {
      hipLaunchKernelGGL(dn_update, dim3(static_cast<uint32_t>((waves + 3) / 4)), dim3(256), 0, st, ua);
      if ((rc = hip_check(hipGetLastError(), "dn_update launch"))) return rc;
      if (p + 1 < npan) {
        uint8_t* tmp = X; X = Y; Y = tmp;
        PanelArgs pa = panel_args(p + 1);
        hipLaunchKernelGGL(dn_panel_ra, dim3(G), dim3(threads), 0, st, pa);
        if ((rc = hip_check(hipGetLastError(), "dn_panel launch"))) return rc;
        continue;
      }
    }
    uint8_t* tmp = X; X = Y; Y = tmp;
  }
  *Xout = X;
  *np_out = np;
  return NTC_GPU_OK;
}

int copy_ok(ntc_gf256_engine* e, uint32_t G, uint8_t* ok, hipStream_t st)
{
  if (!ok) return NTC_GPU_OK;
  return hip_check(hipMemcpyAsync(ok, e->dn_ok, G, hipMemcpyDeviceToDevice, st), "copy ok flags");
}

}  // namespace

extern "C" {

int ntc_gf256_dense_invert_batch(ntc_gf256_engine* e, uint32_t G, uint32_t n, const uint8_t* mat,
                                 uint8_t* inv, uint8_t* ok, void* stream)
{
  if (!e || !mat || !inv) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || n == 0) return fail(NTC_GPU_EINVAL, "G and n must be > 0");
  if (n > kMaxN) return fail(NTC_GPU_EUNSUPPORTED, "dense inversion supports n <= 1024");
  if (G > 65535) return fail(NTC_GPU_EUNSUPPORTED, "G > 65535");
  (void)hipSetDevice(e->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint8_t* X;
  uint32_t np;
  int rc = dense_invert(e, G, n, mat, st, &X, &np);
  if (rc) return rc;
  hipLaunchKernelGGL(dn_gather_inv, dim3(n, G), dim3(256), 0, st, n, np, X,
                     static_cast<const uint32_t*>(e->dn_piv), static_cast<const uint8_t*>(e->dn_ok), inv);
  if ((rc = hip_check(hipGetLastError(), "dn_gather_inv launch"))) return rc;
  return copy_ok(e, G, ok, st);
}

int ntc_gf256_dense_encode_batch(ntc_gf256_engine* e, uint32_t G, uint32_t k, uint32_t r,
                                 uint32_t stride, const uint8_t* mat, const uint8_t* src,
                                 uint8_t* rep, void* stream)
{
  if (!e || !mat || !src || !rep) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || k == 0 || r == 0) return fail(NTC_GPU_EINVAL, "G, k and r must be > 0");
  if (G > 65535) return fail(NTC_GPU_EUNSUPPORTED, "G > 65535");
  (void)hipSetDevice(e->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint32_t pitch = ntc_gf256_coef_pitch(r);
  int rc = ensure_buf(e, &e->dn_coef, &e->dn_coef_cap, static_cast<size_t>(G) * k * pitch + 64, "hipMalloc dense coef");
  if (rc) return rc;
  // combine wants coef[g][i][j] (input-major): the transpose of mat[g][j][i]
  {
    KernelTimer kt(e, NTC_GF256_K_DENSE, st, true);
    hipExtLaunchKernelGGL(dn_transpose, dim3((k + 63) / 64, (pitch + 63) / 64, G), dim3(256), 0, st,
                          kt.start(), kt.stop(), 0, r, k, pitch, mat, static_cast<uint8_t*>(e->dn_coef));
  }
  if ((rc = hip_check(hipGetLastError(), "dn_transpose launch"))) return rc;
  return ntc_gf256_combine_batch(e, G, k, r, stride, src, static_cast<const uint8_t*>(e->dn_coef), rep, stream);
}

int ntc_gf256_dense_decode_batch(ntc_gf256_engine* e, uint32_t G, uint32_t n, uint32_t stride,
                                 const uint8_t* mat, const uint8_t* rep, uint8_t* out, uint8_t* ok,
                                 void* stream)
{
  if (!e || !mat || !rep || !out) return fail(NTC_GPU_EINVAL, "NULL argument");
  if (G == 0 || n == 0) return fail(NTC_GPU_EINVAL, "G and n must be > 0");
  if (n > kMaxN) return fail(NTC_GPU_EUNSUPPORTED, "dense decoding supports n <= 1024");
  if (G > 65535) return fail(NTC_GPU_EUNSUPPORTED, "G > 65535");
  if (stride == 0 || stride % 16 != 0) return fail(NTC_GPU_EINVAL, "stride must be a positive multiple of 16");
  (void)hipSetDevice(e->device);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const uint8_t* X;
  uint32_t np;
  const uint32_t pitch = ntc_gf256_coef_pitch(n);
  int rc;
  {   // timing log: the inversion and the coefficient layout as one NTC_GF256_K_DENSE entry
    KernelTimer kt(e, NTC_GF256_K_DENSE, st);
    if ((rc = dense_invert(e, G, n, mat, st, &X, &np))) return rc;
  // M^-1 rows into the Y buffer (free after the last swap), then transposed into combine layout:
  // out[g][t] = sum_i inv[t][i] * rep[g][i]  ->  coef[g][i][t] = inv[t][i]
  uint8_t* invbuf = static_cast<uint8_t*>(X == e->dn_x ? e->dn_y : e->dn_x);
  hipLaunchKernelGGL(dn_gather_inv, dim3(n, G), dim3(256), 0, st, n, np, X,
                     static_cast<const uint32_t*>(e->dn_piv), static_cast<const uint8_t*>(e->dn_ok), invbuf);
  if ((rc = hip_check(hipGetLastError(), "dn_gather_inv launch"))) return rc;
  if ((rc = ensure_buf(e, &e->dn_coef, &e->dn_coef_cap, static_cast<size_t>(G) * n * pitch + 64, "hipMalloc dense coef"))) return rc;
  hipLaunchKernelGGL(dn_transpose, dim3((n + 63) / 64, (pitch + 63) / 64, G), dim3(256), 0, st, n, n,
                     pitch, invbuf, static_cast<uint8_t*>(e->dn_coef));
  if ((rc = hip_check(hipGetLastError(), "dn_transpose launch"))) return rc;
  }
  if ((rc = ntc_gf256_combine_batch(e, G, n, n, stride, rep, static_cast<const uint8_t*>(e->dn_coef), out, stream))) return rc;
  return copy_ok(e, G, ok, st);
}

}  // extern "C"
