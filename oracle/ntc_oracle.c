/*
 * ntc_oracle.c -- TEST INFRASTRUCTURE ONLY (see ntc_oracle.h).
 *
 * A plain-C restatement of ahamez/netcode's GF(2^8) network-coding path.  Every function cites
 * the reference file:line it follows (paths relative to /root/reference).  Nothing here is
 * shipped: the product is netcode_amd/ + libntc_gf256.so, which never links this file.
 */
#define _GNU_SOURCE
#include "ntc_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ============================================================ GF(2^8), polynomial 0x11D ==== */
/* gf-complete's w=8 default polynomial (galois_field.hh:40 gf_init_easy(&gf, 8)). */

static uint8_t g_exp[512];
static uint8_t g_log[256];
static uint8_t g_mul[256][256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void gf_init_tables(void)
{
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    g_exp[i] = (uint8_t)x;
    g_exp[i + 255] = (uint8_t)x;
    g_log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  g_exp[510] = g_exp[0];
  g_exp[511] = g_exp[1];
  g_log[0] = 0;
  for (int a = 0; a < 256; ++a)
    for (int b = 0; b < 256; ++b)
      g_mul[a][b] = (a == 0 || b == 0) ? 0 : g_exp[g_log[a] + g_log[b]];
}

static inline void gf_init(void) { pthread_once(&g_once, gf_init_tables); }

uint8_t or_gf_mul(uint8_t a, uint8_t b) { gf_init(); return g_mul[a][b]; }

/* ------------------------------------------------ GF(2^w), w in {4, 8, 16, 32} (galois_field.hh) */
/* galois_field.hh:35-44 gf_init_easy(&gf, w): gf-complete's default fields -- primitive
 * polynomials 0x13 (w=4), 0x11D (w=8), 0x1100B (w=16), 0x400007 (+x^32, w=32).  gf-complete is not
 * in /root/reference (no version pin); the polynomials are its published defaults, so for w != 8
 * field bytes are "parity unpinned" against the reference and pinned by field invariants only.
 * The field in use is per thread (the public encoder/decoder entry points select their own). */
static __thread int g_w = 8;
void or_set_field(int w) { g_w = w; }
int or_field(void) { return g_w; }

static uint64_t fw_poly(int w)
{
  return w == 4 ? 0x13u : w == 8 ? 0x11Du : w == 16 ? 0x1100Bu : 0x100400007ull;
}

/* carry-less product reduced by the field polynomial */
uint32_t or_fw_mul(int w, uint32_t a, uint32_t b)
{
  if (a == 0 || b == 0) return 0;
  if (w == 8) { gf_init(); return g_mul[a & 0xFF][b & 0xFF]; }
  uint64_t r = 0;
  for (int i = 0; i < w; ++i)
    if ((b >> i) & 1u) r ^= (uint64_t)a << i;
  const uint64_t p = fw_poly(w);
  for (int i = 2 * w - 2; i >= w; --i)
    if ((r >> i) & 1u) r ^= p << (i - w);
  return (uint32_t)r;
}

/* galois_field.hh:133-139 divide.w32(1, c) = c^(2^w - 2) */
uint32_t or_fw_inv(int w, uint32_t a)
{
  uint32_t res = 1, base = a;
  uint64_t e = (w == 32 ? 0xFFFFFFFFull : ((1ull << w) - 1)) - 1;
  while (e) {
    if (e & 1) res = or_fw_mul(w, res, base);
    base = or_fw_mul(w, base, base);
    e >>= 1;
  }
  return res;
}

/* galois_field.hh:143-158: uint32 arithmetic with wraparound; % (2^w - 1) + 1 for w < 32, the raw
 * product (0 -> 1) for w = 32. */
uint32_t or_fw_coefficient(int w, uint32_t repair_id, uint32_t src_id)
{
  const uint32_t res = ((repair_id + 1u) + (src_id + 1u)) * (repair_id + 1u);
  if (w == 32) return res == 0 ? 1u : res;
  return res % ((1u << w) - 1u) + 1u;
}

/* multiply_region.w32 semantics per w: w=4 every nibble, w=8 every byte, w=16 / w=32 every
 * little-endian 16- / 32-bit word.  A trailing partial word reads missing bytes as zero and only
 * the bytes inside `len` are written. */
void or_fw_region(int w, const uint8_t* src, uint8_t* dst, size_t len, uint32_t c, int add)
{
  if (w == 4) {
    for (size_t i = 0; i < len; ++i) {
      const uint32_t lo = or_fw_mul(4, c, src[i] & 15u), hi = or_fw_mul(4, c, src[i] >> 4);
      const uint8_t v = (uint8_t)((hi << 4) | lo);
      dst[i] = add ? (uint8_t)(dst[i] ^ v) : v;
    }
    return;
  }
  if (w == 8) {
    gf_init();
    const uint8_t* row = g_mul[c & 0xFF];
    for (size_t i = 0; i < len; ++i) dst[i] = add ? (uint8_t)(dst[i] ^ row[src[i]]) : row[src[i]];
    return;
  }
  const size_t wb = (size_t)w / 8;
  for (size_t i = 0; i < len; i += wb) {
    uint32_t x = 0;
    for (size_t b = 0; b < wb && i + b < len; ++b) x |= (uint32_t)src[i + b] << (8 * b);
    const uint32_t v = or_fw_mul(w, c, x);
    for (size_t b = 0; b < wb && i + b < len; ++b) {
      const uint8_t o = (uint8_t)(v >> (8 * b));
      dst[i + b] = add ? (uint8_t)(dst[i + b] ^ o) : o;
    }
  }
}

/* galois_field.hh:96-120: w <= 8 codes the u16 as a 2-byte region (native byte order); w = 16 a
 * scalar product; w = 32 the GF(2^32) product truncated to 16 bits (:118). */
uint16_t or_fw_multiply_size(int w, uint16_t size, uint32_t c)
{
  if (size == 0 || c == 0) return 0;
  if (w <= 8) {
    uint8_t in[2] = {(uint8_t)size, (uint8_t)(size >> 8)}, out[2];
    or_fw_region(w, in, out, 2, c, 0);
    return (uint16_t)(out[0] | (out[1] << 8));
  }
  return (uint16_t)or_fw_mul(w, size, c);
}

uint32_t or_gf_inv(uint32_t a)
{
  /* galois_field.hh:133-139: divide.w32(1, c) */
  if (g_w != 8) return or_fw_inv(g_w, a);
  gf_init();
  return g_exp[(255 - g_log[a & 0xFF]) % 255];
}

/* galois_field.hh:143-158 (field of this thread; w = 8: % 255 + 1). */
uint32_t or_coefficient(uint32_t repair_id, uint32_t src_id)
{
  return or_fw_coefficient(g_w, repair_id, src_id);
}

static int g_simd = 0;   /* CPU-baseline mode: 1 = AVX2 split-nibble region ops, 2 = GFNI (if present) */
static void muladd_dispatch(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c);

void or_set_simd(int on) { gf_init(); g_simd = on; }

/* galois_field.hh:65-75: multiply_region.w32(..., add = 0) */
void or_region_mul(const uint8_t* src, uint8_t* dst, size_t len, uint32_t c)
{
  gf_init();
  if (g_w != 8) { or_fw_region(g_w, src, dst, len, c, 0); return; }
  if (g_simd) { memset(dst, 0, len); muladd_dispatch(src, dst, len, (uint8_t)c); return; }
  const uint8_t* row = g_mul[c & 0xFF];
  for (size_t i = 0; i < len; ++i) dst[i] = row[src[i]];
}

/* galois_field.hh:83-92: multiply_region.w32(..., add = 1) */
void or_region_muladd(const uint8_t* src, uint8_t* dst, size_t len, uint32_t c)
{
  gf_init();
  if (g_w != 8) { or_fw_region(g_w, src, dst, len, c, 1); return; }
  if (g_simd) { muladd_dispatch(src, dst, len, (uint8_t)c); return; }
  const uint8_t* row = g_mul[c & 0xFF];
  for (size_t i = 0; i < len; ++i) dst[i] ^= row[src[i]];
}

/* galois_field.hh:96-120 */
uint16_t or_multiply_size(uint16_t size, uint32_t c)
{
  return or_fw_multiply_size(g_w, size, c);
}

static inline uint32_t gf_mul32(uint32_t x, uint32_t y)
{
  /* galois_field.hh:123-130 */
  return or_fw_mul(g_w, x, y);
}

/* Dense codes (config 5 extension): plain region MACs over a caller-chosen matrix. */
void or_dense_encode(uint32_t k, uint32_t r, size_t stride, const uint8_t* mat, const uint8_t* src,
                     uint8_t* rep)
{
  for (uint32_t j = 0; j < r; ++j) {
    uint8_t* out = rep + (size_t)j * stride;
    memset(out, 0, stride);
    for (uint32_t i = 0; i < k; ++i)
      if (mat[(size_t)j * k + i]) or_region_muladd(src + (size_t)i * stride, out, stride, mat[(size_t)j * k + i]);
  }
}

long or_dense_decode(uint32_t n, size_t stride, const uint8_t* mat, const uint8_t* rep, uint8_t* out,
                     uint8_t* inv)
{
  const size_t nn = (size_t)n * n;
  uint32_t* m = (uint32_t*)malloc(nn * sizeof(uint32_t));
  uint32_t* mi = (uint32_t*)malloc(nn * sizeof(uint32_t));
  for (size_t e = 0; e < nn; ++e) m[e] = mat[e];
  /* or_invert works on storage rows; the inverse of the row-major matrix comes out row-major */
  const long fail = or_invert(m, mi, n);
  memset(out, 0, (size_t)n * stride);
  if (inv) for (size_t e = 0; e < nn; ++e) inv[e] = fail < 0 ? (uint8_t)mi[e] : 0;
  if (fail < 0)
    for (uint32_t t = 0; t < n; ++t)
      for (uint32_t i = 0; i < n; ++i)
        if (mi[(size_t)t * n + i]) or_region_muladd(rep + (size_t)i * stride, out + (size_t)t * stride, stride, (uint8_t)mi[(size_t)t * n + i]);
  free(m);
  free(mi);
  return fail;
}

/* invert_matrix.cc:9-128 (jerasure_invert_matrix order; storage rows are matrix columns). */
long or_invert(uint32_t* mat, uint32_t* inv, size_t n)
{
  gf_init();
  const size_t cols = n, rows = n;
  for (size_t i = 0; i < rows; ++i)
    for (size_t j = 0; j < cols; ++j)
      inv[j * n + i] = (i == j) ? 1 : 0;             /* inv(i,j), col-major */

  for (size_t i = 0; i < cols; ++i) {
    const size_t row_start = i * cols;
    if (mat[row_start + i] == 0) {                   /* :33-57 row swap */
      size_t j;
      for (j = i + 1; j < rows && mat[cols * j + i] == 0; ++j) {}
      if (j == rows) return (long)(j - 1);           /* :40-44 failure index = rows-1 */
      const size_t rs2 = j * cols;
      for (size_t k = 0; k < cols; ++k) {
        uint32_t t = mat[row_start + k]; mat[row_start + k] = mat[rs2 + k]; mat[rs2 + k] = t;
        t = inv[row_start + k]; inv[row_start + k] = inv[rs2 + k]; inv[rs2 + k] = t;
      }
    }
    const uint32_t tmp = mat[row_start + i];         /* :59-69 normalise */
    if (tmp != 1) {
      const uint32_t inverse = or_gf_inv(tmp);
      for (size_t j = 0; j < cols; ++j) {
        mat[row_start + j] = gf_mul32(mat[row_start + j], inverse);
        inv[row_start + j] = gf_mul32(inv[row_start + j], inverse);
      }
    }
    size_t k = row_start + i;                        /* :71-98 eliminate below */
    for (size_t j = i + 1; j != cols; ++j) {
      k += cols;
      if (mat[k] != 0) {
        const size_t rs2 = cols * j;
        if (mat[k] == 1) {
          for (size_t x = 0; x < cols; ++x) {
            mat[rs2 + x] ^= mat[row_start + x];
            inv[rs2 + x] ^= inv[row_start + x];
          }
        } else {
          const uint32_t mk = mat[k];
          for (size_t x = 0; x < cols; ++x) {
            mat[rs2 + x] ^= gf_mul32(mk, mat[row_start + x]);
            inv[rs2 + x] ^= gf_mul32(mk, inv[row_start + x]);
          }
        }
      }
    }
  }
  for (size_t i = rows - 1;; --i) {                  /* :101-123 back substitution */
    const size_t row_start = i * cols;
    for (size_t j = 0; j < i; ++j) {
      const size_t rs2 = j * cols;
      if (mat[rs2 + i] != 0) {
        const uint32_t tmp2 = mat[rs2 + i];
        mat[rs2 + i] = 0;
        for (size_t k2 = 0; k2 < cols; ++k2)
          inv[rs2 + k2] ^= gf_mul32(tmp2, inv[row_start + k2]);
      }
    }
    if (i == 0) break;
  }
  return -1;
}

/* ==================================================================== AVX2 region MAC ==== */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("avx2")))
static void muladd_avx2(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c)
{
  /* Split-nibble tables (gf-complete SPLIT 8,4 / "pshufb" region multiply). */
  uint8_t lo[16], hi[16];
  for (int t = 0; t < 16; ++t) { lo[t] = g_mul[c][t]; hi[t] = g_mul[c][t << 4]; }
  const __m256i tlo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)lo));
  const __m256i thi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)hi));
  const __m256i m = _mm256_set1_epi8(0x0F);
  size_t i = 0;
  for (; i + 32 <= len; i += 32) {
    const __m256i x = _mm256_loadu_si256((const __m256i*)(src + i));
    const __m256i l = _mm256_shuffle_epi8(tlo, _mm256_and_si256(x, m));
    const __m256i h = _mm256_shuffle_epi8(thi, _mm256_and_si256(_mm256_srli_epi16(x, 4), m));
    __m256i d = _mm256_loadu_si256((const __m256i*)(dst + i));
    d = _mm256_xor_si256(d, _mm256_xor_si256(l, h));
    _mm256_storeu_si256((__m256i*)(dst + i), d);
  }
  const uint8_t* row = g_mul[c];
  for (; i < len; ++i) dst[i] ^= row[src[i]];
}
int or_have_avx2(void) { return __builtin_cpu_supports("avx2"); }

/* GFNI + AVX-512 region MAC (a labelled CPU upper bound, not gf-complete's
 * algorithm).  Multiplication by c is GF(2)-linear on the bits of a byte: y_i = XOR_j M[i][j] x_j
 * with column j = c * 2^j (mod 0x11D); gf2p8affineqb applies such a matrix to 64 bytes at once,
 * taking row i from byte 7-i of the matrix qword.  (gf2p8mulb is fixed to the AES polynomial
 * 0x11B, so it cannot be used for netcode's 0x11D field.) */
__attribute__((target("avx512f,avx512bw,gfni")))
static void muladd_gfni(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c)
{
  uint64_t A = 0;
  for (int i = 0; i < 8; ++i) {
    uint64_t row = 0;
    for (int j = 0; j < 8; ++j) row |= (uint64_t)((g_mul[c][1u << j] >> i) & 1u) << j;
    A |= row << (8 * (7 - i));
  }
  const __m512i a = _mm512_set1_epi64((long long)A);
  size_t i = 0;
  for (; i + 64 <= len; i += 64) {
    const __m512i x = _mm512_loadu_si512((const void*)(src + i));
    const __m512i d = _mm512_loadu_si512((const void*)(dst + i));
    _mm512_storeu_si512((void*)(dst + i), _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(x, a, 0)));
  }
  const uint8_t* row = g_mul[c];
  for (; i < len; ++i) dst[i] ^= row[src[i]];
}
int or_have_gfni(void)
{
  return __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw") &&
         __builtin_cpu_supports("avx512f");
}
#else
int or_have_avx2(void) { return 0; }
int or_have_gfni(void) { return 0; }
#endif

static void muladd_dispatch(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c)
{
#if defined(__x86_64__)
  if (g_simd == 2 && or_have_gfni()) { muladd_gfni(src, dst, len, c); return; }
  if (or_have_avx2()) { muladd_avx2(src, dst, len, c); return; }
#endif
  const uint8_t* row = g_mul[c];
  for (size_t i = 0; i < len; ++i) dst[i] ^= row[src[i]];
}

void or_region_muladd_simd(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c)
{
  gf_init();
  muladd_dispatch(src, dst, len, c);
}

/* ===================================================== generation encode (batch form) ==== */
static void encode_generation_impl(uint32_t k, uint32_t r, uint32_t stride, const uint8_t* src,
                                   const uint16_t* src_len, uint32_t sid_base, uint32_t rid_base,
                                   uint8_t* rep, uint16_t* rep_size, uint16_t* rep_len,
                                   int use_simd)
{
  /* detail/encoder.cc:15-64 per repair; repairs emitted by encoder.hh:162-169, 321-333. */
  gf_init();
  uint16_t max_len = 0;
  for (uint32_t i = 0; i < k; ++i) if (src_len[i] > max_len) max_len = src_len[i];
  for (uint32_t j = 0; j < r; ++j) {
    uint8_t* out = rep + (size_t)j * stride;
    memset(out, 0, stride);                          /* zero_byte_buffer growth, :26 / :45-48 */
    uint16_t esz = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const uint8_t c = (uint8_t)or_coefficient(rid_base + j, sid_base + i);
      const uint8_t* s = src + (size_t)i * stride;
      if (use_simd) or_region_muladd_simd(s, out, src_len[i], c);
      else if (i == 0) or_region_mul(s, out, src_len[i], c);      /* :35 multiply */
      else or_region_muladd(s, out, src_len[i], c);               /* :57 multiply_add */
      esz = (uint16_t)(or_multiply_size(src_len[i], c) ^ esz);    /* :38, :61-62 */
    }
    if (rep_size) rep_size[j] = esz;
    if (rep_len) rep_len[j] = max_len;
  }
}

void or_encode_generation(uint32_t k, uint32_t r, uint32_t stride, const uint8_t* src,
                          const uint16_t* src_len, uint32_t sid_base, uint32_t rid_base,
                          uint8_t* rep, uint16_t* rep_size, uint16_t* rep_len)
{
  encode_generation_impl(k, r, stride, src, src_len, sid_base, rid_base, rep, rep_size, rep_len,
                         0);
}

/* ------------------------------------------------------------------ thread fan-out ------- */
typedef struct {
  int kind; /* 0 encode, 1 decode */
  uint32_t g0, g1, k, r, stride;
  const uint8_t* csrc; uint8_t* src; uint16_t* src_len; const uint16_t* csrc_len;
  const uint8_t* src_mask; const uint8_t* crep; uint8_t* rep; uint16_t* rep_size;
  const uint16_t* crep_size; const uint16_t* rep_len; const uint8_t* rep_mask;
  const uint32_t* sid_base; const uint32_t* rid_base; or_decode_status* st; int use_simd;
} batch_job;

static void decode_generation_impl(uint32_t k, uint32_t r, uint32_t stride, uint8_t* src,
                                   uint16_t* src_len, const uint8_t* src_mask, const uint8_t* rep,
                                   const uint16_t* rep_size, const uint16_t* rep_len,
                                   const uint8_t* rep_mask, uint32_t sid_base, uint32_t rid_base,
                                   or_decode_status* st, int use_simd);

static void* batch_worker(void* p)
{
  batch_job* j = (batch_job*)p;
  for (uint32_t g = j->g0; g < j->g1; ++g) {
    const size_t so = (size_t)g * j->k, ro = (size_t)g * j->r;
    const uint32_t sb = j->sid_base ? j->sid_base[g] : g * j->k;
    const uint32_t rb = j->rid_base ? j->rid_base[g] : g * j->r;
    if (j->kind == 0)
      encode_generation_impl(j->k, j->r, j->stride, j->csrc + so * j->stride, j->csrc_len + so,
                             sb, rb, j->rep + ro * j->stride, j->rep_size + ro, NULL, j->use_simd);
    else
      decode_generation_impl(j->k, j->r, j->stride, j->src + so * j->stride, j->src_len + so,
                             j->src_mask + so, j->crep + ro * j->stride, j->crep_size + ro,
                             j->rep_len ? j->rep_len + ro : NULL, j->rep_mask + ro, sb, rb,
                             j->st + g, j->use_simd);
  }
  return NULL;
}

static void run_batch(batch_job* proto, uint32_t G, int nthreads)
{
  if (nthreads < 1) nthreads = 1;
  if ((uint32_t)nthreads > G) nthreads = (int)(G ? G : 1);
  pthread_t th[256];
  batch_job jobs[256];
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = *proto;
    jobs[t].g0 = (uint32_t)((uint64_t)G * t / nthreads);
    jobs[t].g1 = (uint32_t)((uint64_t)G * (t + 1) / nthreads);
    if (nthreads == 1) batch_worker(&jobs[t]);
    else pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
}

void or_encode_batch(uint32_t G, uint32_t k, uint32_t r, uint32_t stride, const uint8_t* src,
                     const uint16_t* src_len, const uint32_t* sid_base, const uint32_t* rid_base,
                     uint8_t* rep, uint16_t* rep_size, int use_simd, int nthreads)
{
  gf_init();
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 0; j.k = k; j.r = r; j.stride = stride; j.csrc = src; j.csrc_len = src_len;
  j.sid_base = sid_base; j.rid_base = rid_base; j.rep = rep; j.rep_size = rep_size;
  j.use_simd = use_simd;
  run_batch(&j, G, nthreads);
}

/* ================================================= streaming decoder state machine ========= */
/* detail/decoder.{hh,cc} restated with sorted dynamic arrays instead of boost maps. */

typedef struct { uint32_t* v; size_t n, cap; } u32set;        /* sorted, unique */

static size_t u32set_lb(const u32set* s, uint32_t x)
{
  size_t lo = 0, hi = s->n;
  while (lo < hi) { size_t mid = (lo + hi) / 2; if (s->v[mid] < x) lo = mid + 1; else hi = mid; }
  return lo;
}
static int u32set_has(const u32set* s, uint32_t x)
{
  size_t i = u32set_lb(s, x);
  return i < s->n && s->v[i] == x;
}
static void u32set_insert(u32set* s, uint32_t x)
{
  size_t i = u32set_lb(s, x);
  if (i < s->n && s->v[i] == x) return;
  if (s->n == s->cap) { s->cap = s->cap ? 2 * s->cap : 8; s->v = realloc(s->v, s->cap * 4); }
  memmove(s->v + i + 1, s->v + i, (s->n - i) * 4);
  s->v[i] = x; s->n++;
}
static void u32set_erase(u32set* s, uint32_t x)
{
  size_t i = u32set_lb(s, x);
  if (i < s->n && s->v[i] == x) { memmove(s->v + i, s->v + i + 1, (s->n - i - 1) * 4); s->n--; }
}
static void u32set_free(u32set* s) { free(s->v); s->v = NULL; s->n = s->cap = 0; }
static void u32set_copy(u32set* d, const u32set* s)
{
  d->n = s->n; d->cap = s->n ? s->n : 1; d->v = malloc(d->cap * 4);
  memcpy(d->v, s->v, s->n * 4);
}

typedef struct { uint32_t id; uint16_t len; uint8_t* data; } dsrc;
typedef struct { uint32_t id; u32set ids; uint16_t esz; uint16_t symsz; uint8_t* sym; } drep;
typedef struct { uint32_t sid; u32set rids; } dmiss;

typedef struct {
  int in_order;
  uint32_t first_missing;
  u32set ordered;                        /* ids of sources waiting for in-order delivery */
  dsrc* src; size_t nsrc, capsrc;        /* sorted by id */
  drep* rep; size_t nrep, caprep;        /* sorted by id */
  dmiss* miss; size_t nmiss, capmiss;    /* sorted by sid */
  int has_last; uint32_t last_id;
  size_t nb_useless, nb_failed, nb_decoded;
  void (*cb)(void*, const dsrc*);
  void* cbctx;
} dec_core;

static size_t src_lb(const dec_core* d, uint32_t id)
{
  size_t lo = 0, hi = d->nsrc;
  while (lo < hi) { size_t m = (lo + hi) / 2; if (d->src[m].id < id) lo = m + 1; else hi = m; }
  return lo;
}
static dsrc* src_find(dec_core* d, uint32_t id)
{
  size_t i = src_lb(d, id);
  return (i < d->nsrc && d->src[i].id == id) ? &d->src[i] : NULL;
}
static size_t rep_lb(const dec_core* d, uint32_t id)
{
  size_t lo = 0, hi = d->nrep;
  while (lo < hi) { size_t m = (lo + hi) / 2; if (d->rep[m].id < id) lo = m + 1; else hi = m; }
  return lo;
}
static drep* rep_find(dec_core* d, uint32_t id)
{
  size_t i = rep_lb(d, id);
  return (i < d->nrep && d->rep[i].id == id) ? &d->rep[i] : NULL;
}
static size_t miss_lb(const dec_core* d, uint32_t id)
{
  size_t lo = 0, hi = d->nmiss;
  while (lo < hi) { size_t m = (lo + hi) / 2; if (d->miss[m].sid < id) lo = m + 1; else hi = m; }
  return lo;
}
static dmiss* miss_find(dec_core* d, uint32_t id)
{
  size_t i = miss_lb(d, id);
  return (i < d->nmiss && d->miss[i].sid == id) ? &d->miss[i] : NULL;
}
static dmiss* miss_get(dec_core* d, uint32_t id)     /* operator[] */
{
  size_t i = miss_lb(d, id);
  if (i < d->nmiss && d->miss[i].sid == id) return &d->miss[i];
  if (d->nmiss == d->capmiss) {
    d->capmiss = d->capmiss ? 2 * d->capmiss : 16;
    d->miss = realloc(d->miss, d->capmiss * sizeof(dmiss));
  }
  memmove(d->miss + i + 1, d->miss + i, (d->nmiss - i) * sizeof(dmiss));
  memset(&d->miss[i], 0, sizeof(dmiss));
  d->miss[i].sid = id;
  d->nmiss++;
  return &d->miss[i];
}
static void miss_erase_at(dec_core* d, size_t i)
{
  u32set_free(&d->miss[i].rids);
  memmove(d->miss + i, d->miss + i + 1, (d->nmiss - i - 1) * sizeof(dmiss));
  d->nmiss--;
}
static void rep_erase_at(dec_core* d, size_t i)
{
  u32set_free(&d->rep[i].ids);
  free(d->rep[i].sym);
  memmove(d->rep + i, d->rep + i + 1, (d->nrep - i - 1) * sizeof(drep));
  d->nrep--;
}
static dsrc* src_insert(dec_core* d, dsrc s)
{
  size_t i = src_lb(d, s.id);
  if (d->nsrc == d->capsrc) {
    d->capsrc = d->capsrc ? 2 * d->capsrc : 64;
    d->src = realloc(d->src, d->capsrc * sizeof(dsrc));
  }
  memmove(d->src + i + 1, d->src + i, (d->nsrc - i) * sizeof(dsrc));
  d->src[i] = s;
  d->nsrc++;
  return &d->src[i];
}
static drep* rep_insert(dec_core* d, drep r)
{
  size_t i = rep_lb(d, r.id);
  if (d->nrep == d->caprep) {
    d->caprep = d->caprep ? 2 * d->caprep : 16;
    d->rep = realloc(d->rep, d->caprep * sizeof(drep));
  }
  memmove(d->rep + i + 1, d->rep + i, (d->nrep - i) * sizeof(drep));
  d->rep[i] = r;
  d->nrep++;
  return &d->rep[i];
}

static void deliver_id(dec_core* d, uint32_t id)
{
  dsrc* s = src_find(d, id);
  if (s) d->cb(d->cbctx, s);
}

/* detail/decoder.cc:570-591 */
static void flush_ordered_sources(dec_core* d)
{
  size_t i = u32set_lb(&d->ordered, d->first_missing);
  if (i < d->ordered.n && d->ordered.v[i] == d->first_missing) {
    for (;;) {
      const uint32_t id = d->ordered.v[i];
      deliver_id(d, id);
      memmove(d->ordered.v + i, d->ordered.v + i + 1, (d->ordered.n - i - 1) * 4);
      d->ordered.n--;
      d->first_missing += 1;
      if (i == d->ordered.n || d->ordered.v[i] > d->first_missing) break;
    }
  }
}

/* detail/decoder.cc:393-408 */
static void remove_source_data_from_repair(const dsrc* s, drep* r)
{
  const uint32_t c = or_coefficient(r->id, s->id);
  r->esz = (uint16_t)(or_multiply_size(s->len, c) ^ r->esz);
  or_region_muladd(s->data, r->sym, s->len, c);
}

/* detail/decoder.cc:156-178 */
static dsrc create_source_from_repair(dec_core* d, const drep* r)
{
  const uint32_t sid = r->ids.v[0];
  const uint32_t inv = or_gf_inv(or_coefficient(r->id, sid));
  const uint16_t sz = or_multiply_size(r->esz, inv);
  dsrc s;
  s.id = sid; s.len = sz;
  s.data = calloc((size_t)sz + 16, 1);
  /* :173 multiply(r.symbol(), src.symbol(), src_sz, inv) -- reads src_sz bytes of the repair
   * symbol; the decoder_repair's packet is at least that long in every reachable state. */
  const size_t n = sz <= r->symsz ? sz : r->symsz;
  or_region_mul(r->sym, s.data, n, inv);
  d->nb_decoded += 1;
  return s;
}

static void add_source_recursive(dec_core* d, dsrc s);

/* detail/decoder.cc:182-191 */
static void remove_source_from_repair(const dsrc* s, drep* r)
{
  remove_source_data_from_repair(s, r);
  u32set_erase(&r->ids, s->id);
}

/* detail/decoder.cc:249-337 */
static void add_source_recursive(dec_core* d, dsrc s)
{
  if (!d->in_order) {
    d->cb(d->cbctx, &s);
  } else if (s.id == d->first_missing) {
    d->cb(d->cbctx, &s);
    d->first_missing += 1;
    flush_ordered_sources(d);
  }

  /* :265-277 remove this source from all repairs that encode it */
  {
    size_t mi = miss_lb(d, s.id);
    if (mi < d->nmiss && d->miss[mi].sid == s.id) {
      u32set rids;
      u32set_copy(&rids, &d->miss[mi].rids);
      for (size_t t = 0; t < rids.n; ++t) {
        drep* r = rep_find(d, rids.v[t]);
        if (r) remove_source_from_repair(&s, r);
      }
      u32set_free(&rids);
      mi = miss_lb(d, s.id);
      miss_erase_at(d, mi);
    }
  }

  /* :279-325 peel repairs that encode exactly one missing source */
  size_t mi = 0;
  while (mi < d->nmiss) {
    dmiss* m = &d->miss[mi];
    if (m->rids.n == 1) {
      drep* r = rep_find(d, m->rids.v[0]);
      if (r && r->ids.n == 1) {
        dsrc dec = create_source_from_repair(d, r);
        const uint32_t cur = m->sid;
        rep_erase_at(d, (size_t)(r - d->rep));
        miss_erase_at(d, mi);
        add_source_recursive(d, dec);
        /* The reference continues from the iterator returned by erase(); re-find it by key
         * (identical whenever the reference's iterator is still valid). */
        mi = miss_lb(d, cur);
        continue;
      }
    }
    ++mi;
  }

  const uint32_t sid = s.id;
  src_insert(d, s);
  if (d->in_order && sid > d->first_missing) u32set_insert(&d->ordered, sid);
}

/* detail/decoder.cc:341-389 */
static void drop_outdated(dec_core* d, uint32_t id)
{
  d->has_last = 1;
  d->last_id = id;
  for (size_t i = 0; i < d->nrep;) {
    drep* r = &d->rep[i];
    if (id > r->ids.v[0]) {
      for (size_t t = 0; t < r->ids.n; ++t) {
        dmiss* m = miss_find(d, r->ids.v[t]);
        if (m) u32set_erase(&m->rids, r->id);
      }
      rep_erase_at(d, i);
    } else {
      ++i;
    }
  }
  if (d->in_order) {
    while (d->ordered.n && d->ordered.v[0] < id) {
      const uint32_t oid = d->ordered.v[0];
      deliver_id(d, oid);
      memmove(d->ordered.v, d->ordered.v + 1, (d->ordered.n - 1) * 4);
      d->ordered.n--;
    }
    if (d->first_missing < id) d->first_missing = id;
    flush_ordered_sources(d);
  }
  const size_t ns = src_lb(d, id);
  for (size_t i = 0; i < ns; ++i) free(d->src[i].data);
  memmove(d->src, d->src + ns, (d->nsrc - ns) * sizeof(dsrc));
  d->nsrc -= ns;
  const size_t nm = miss_lb(d, id);
  for (size_t i = 0; i < nm; ++i) u32set_free(&d->miss[i].rids);
  memmove(d->miss, d->miss + nm, (d->nmiss - nm) * sizeof(dmiss));
  d->nmiss -= nm;
}

/* detail/decoder.cc:412-566 */
static int attempt_full_decoding(dec_core* d)
{
  if (d->nrep == 0 || d->nmiss == 0) return 0;
  if (d->nmiss > d->nrep) return 0;
  const size_t n = d->nrep;
  uint32_t* coef = malloc(n * n * 4);
  uint32_t* inv = malloc(n * n * 4);
  for (size_t col = 0; col < n; ++col)              /* :430-443 coefficients(row, col) */
    for (size_t row = 0; row < n; ++row)
      coef[col * n + row] = u32set_has(&d->rep[col].ids, d->miss[row].sid)
                          ? or_coefficient(d->rep[col].id, d->miss[row].sid) : 0u;
  const long fail = or_invert(coef, inv, n);
  if (fail >= 0) {                                   /* :448-468 */
    d->nb_failed += 1;
    drep* r = &d->rep[fail];
    for (size_t t = 0; t < r->ids.n; ++t) {
      dmiss* m = miss_get(d, r->ids.v[t]);
      u32set_erase(&m->rids, r->id);
      r = &d->rep[fail];                             /* miss_get may not move reps; re-read */
    }
    rep_erase_at(d, (size_t)fail);
    free(coef); free(inv);
    return 1;
  }
  /* :480-559 */
  const size_t nm = d->nmiss;
  uint32_t* mids = malloc(nm * 4);
  for (size_t s = 0; s < nm; ++s) mids[s] = d->miss[s].sid;
  for (size_t sc = 0; sc < nm; ++sc) {
    uint16_t sz = 0;
    for (size_t rr = 0; rr < n; ++rr) {
      const uint32_t c = inv[sc * n + rr];           /* m_inv(repair_row, src_col) */
      if (c != 0) sz = (uint16_t)(or_multiply_size(d->rep[rr].esz, c) ^ sz);
    }
    dsrc s;
    s.id = mids[sc]; s.len = sz;
    s.data = calloc((size_t)sz + 16, 1);
    size_t rr = 0;
    uint32_t c = 0;
    for (; rr < n; ++rr) { c = inv[sc * n + rr]; if (c != 0) break; }
    size_t len = sz < d->rep[rr].symsz ? sz : d->rep[rr].symsz;
    or_region_mul(d->rep[rr].sym, s.data, len, c);
    for (++rr; rr < n; ++rr) {
      c = inv[sc * n + rr];
      if (c != 0) {
        len = sz < d->rep[rr].symsz ? sz : d->rep[rr].symsz;
        or_region_muladd(d->rep[rr].sym, s.data, len, c);
      }
    }
    const uint32_t sid = s.id;
    src_insert(d, s);
    if (!d->in_order) {
      deliver_id(d, sid);
    } else if (sid == d->first_missing) {
      deliver_id(d, sid);
      d->first_missing += 1;
      flush_ordered_sources(d);
    } else {
      u32set_insert(&d->ordered, sid);
    }
  }
  d->nb_decoded += nm;
  while (d->nrep) rep_erase_at(d, d->nrep - 1);     /* :564-565 */
  while (d->nmiss) miss_erase_at(d, d->nmiss - 1);
  free(mids); free(coef); free(inv);
  return 2;
}

/* detail/decoder.cc:33-50 */
static void core_add_source(dec_core* d, uint32_t id, const uint8_t* data, uint16_t len)
{
  if (d->has_last && id < d->last_id) return;
  if (src_find(d, id)) return;
  dsrc s;
  s.id = id; s.len = len;
  s.data = malloc((size_t)len + 16);
  memcpy(s.data, data, len);
  add_source_recursive(d, s);
  attempt_full_decoding(d);
}

/* detail/decoder.cc:54-152.  `ids` must be sorted & unique (flat_set). Returns 0 dropped
 * (outdated / duplicate / useless), 1 stored/decoded. */
static int core_add_repair(dec_core* d, uint32_t id, const uint32_t* ids, size_t nids,
                           uint16_t esz, const uint8_t* sym, uint16_t symsz)
{
  const uint32_t last = ids[nids - 1];
  if (d->has_last && last < d->last_id) return 0;
  if (rep_find(d, id)) return 0;
  drop_outdated(d, ids[0]);
  int useless = 1;
  for (size_t t = 0; t < nids; ++t) if (!src_find(d, ids[t])) { useless = 0; break; }
  if (useless) { d->nb_useless += 1; return 0; }

  drep nr;
  nr.id = id; nr.esz = esz; nr.symsz = symsz;
  memset(&nr.ids, 0, sizeof nr.ids);
  for (size_t t = 0; t < nids; ++t) u32set_insert(&nr.ids, ids[t]);
  nr.sym = malloc((size_t)symsz + 16);
  memcpy(nr.sym, sym, symsz);
  drep* r = rep_insert(d, nr);

  /* :102-130 reverse loop over source ids */
  for (size_t t = r->ids.n; t-- > 0;) {
    const uint32_t sid = r->ids.v[t];
    dsrc* s = src_find(d, sid);
    if (s) {
      remove_source_data_from_repair(s, r);
      memmove(r->ids.v + t, r->ids.v + t + 1, (r->ids.n - t - 1) * 4);
      r->ids.n--;
    } else {
      dmiss* m = miss_get(d, sid);
      u32set_insert(&m->rids, id);
    }
    r = rep_find(d, id);
  }
  if (r->ids.n == 1) {                               /* :134-149 */
    dsrc s = create_source_from_repair(d, r);
    const size_t mi = miss_lb(d, s.id);
    if (mi < d->nmiss && d->miss[mi].sid == s.id) miss_erase_at(d, mi);
    rep_erase_at(d, (size_t)(r - d->rep));
    add_source_recursive(d, s);
    return 1;
  }
  attempt_full_decoding(d);
  return 1;
}

static void core_init(dec_core* d, int in_order, void (*cb)(void*, const dsrc*), void* ctx)
{
  memset(d, 0, sizeof *d);
  d->in_order = in_order;
  d->cb = cb;
  d->cbctx = ctx;
}

static void core_free(dec_core* d)
{
  for (size_t i = 0; i < d->nsrc; ++i) free(d->src[i].data);
  while (d->nrep) rep_erase_at(d, d->nrep - 1);
  while (d->nmiss) miss_erase_at(d, d->nmiss - 1);
  free(d->src); free(d->rep); free(d->miss);
  u32set_free(&d->ordered);
}

/* ============================================ the streaming decoder as an object (tests) ==== */
/* detail::decoder (detail/decoder.hh:21-193) over dec_core, for tests/oracle_surface: the reference
 * Catch suites drive it through their own accessors.  Every call runs in the object's field. */
struct or_dcore { dec_core core; int w; or_source_fn cb; void* ctx; };

static void dcore_deliver(void* ctx, const dsrc* s)
{
  or_dcore* o = (or_dcore*)ctx;
  if (o->cb) o->cb(o->ctx, s->id, s->data, s->len);
}

or_dcore* or_dcore_new(int w, int in_order, or_source_fn cb, void* ctx)
{
  gf_init();
  or_dcore* o = calloc(1, sizeof *o);
  o->w = w; o->cb = cb; o->ctx = ctx;
  core_init(&o->core, in_order, dcore_deliver, o);
  return o;
}
void or_dcore_free(or_dcore* o) { if (o) { core_free(&o->core); free(o); } }

#define DCORE_FIELD(o, stmt) do { const int old_ = g_w; g_w = (o)->w; stmt; g_w = old_; } while (0)

void or_dcore_add_source(or_dcore* o, uint32_t id, const uint8_t* data, uint16_t len)
{
  DCORE_FIELD(o, core_add_source(&o->core, id, data, len));
}
void or_dcore_add_repair(or_dcore* o, uint32_t id, const uint32_t* ids, size_t n, uint16_t esz,
                         const uint8_t* sym, uint16_t symsz)
{
  if (n == 0) return;
  DCORE_FIELD(o, core_add_repair(&o->core, id, ids, n, esz, sym, symsz));
}

/* decoder.cc:156-178 on a stand-alone one-source repair (bumps nb_decoded).  out receives the
 * multiply_size(esz, inv) bytes of the source; returns that size. */
uint16_t or_dcore_create_source_from_repair(or_dcore* o, uint32_t rid, uint32_t sid, uint16_t esz,
                                            const uint8_t* sym, uint16_t symsz, uint8_t* out)
{
  drep r;
  memset(&r, 0, sizeof r);
  r.id = rid; r.esz = esz; r.symsz = symsz;
  r.sym = (uint8_t*)sym;
  u32set_insert(&r.ids, sid);
  dsrc s;
  DCORE_FIELD(o, s = create_source_from_repair(&o->core, &r));
  u32set_free(&r.ids);
  memcpy(out, s.data, s.len);
  free(s.data);
  return s.len;
}

/* decoder.cc:182-191 + 393-408 on a stand-alone repair: subtract the source from sym / esz (the
 * caller drops sid from the repair's id list). */
void or_dcore_remove_source_from_repair(or_dcore* o, uint32_t sid, const uint8_t* sdata, uint16_t slen,
                                        uint32_t rid, uint16_t* esz, uint8_t* sym)
{
  dsrc s = {sid, slen, (uint8_t*)sdata};
  drep r;
  memset(&r, 0, sizeof r);
  r.id = rid; r.esz = *esz; r.sym = sym;
  DCORE_FIELD(o, remove_source_data_from_repair(&s, &r));
  *esz = r.esz;
}

size_t or_dcore_count(const or_dcore* o, int which)
{
  switch (which) {
    case 0: return o->core.nsrc;
    case 1: return o->core.nrep;
    case 2: return o->core.nmiss;
    case 3: return o->core.nb_decoded;
    case 4: return o->core.nb_failed;
    case 5: return o->core.nb_useless;
    default: return 0;
  }
}
uint32_t or_dcore_source(const or_dcore* o, size_t i, const uint8_t** data, uint16_t* len)
{
  *data = o->core.src[i].data; *len = o->core.src[i].len;
  return o->core.src[i].id;
}
uint32_t or_dcore_repair(const or_dcore* o, size_t i, const uint32_t** ids, size_t* n, uint16_t* esz,
                         const uint8_t** sym, uint16_t* symsz)
{
  const drep* r = &o->core.rep[i];
  *ids = r->ids.v; *n = r->ids.n; *esz = r->esz; *sym = r->sym; *symsz = r->symsz;
  return r->id;
}
uint32_t or_dcore_missing(const or_dcore* o, size_t i, const uint32_t** rids, size_t* n)
{
  *rids = o->core.miss[i].rids.v; *n = o->core.miss[i].rids.n;
  return o->core.miss[i].sid;
}

/* ===================================================== generation decode (batch form) ====== */
typedef struct { uint8_t* src; uint32_t stride, sid_base, k; uint16_t* src_len; } gen_sink;

static void gen_deliver(void* ctx, const dsrc* s)
{
  gen_sink* g = (gen_sink*)ctx;
  const uint32_t slot = s->id - g->sid_base;
  if (slot >= g->k) return;
  uint8_t* out = g->src + (size_t)slot * g->stride;
  const size_t n = s->len < g->stride ? s->len : g->stride;
  if (out != s->data) {
    memmove(out, s->data, n);
    memset(out + n, 0, g->stride - n);
  }
  g->src_len[slot] = s->len;
}

static void decode_generation_impl(uint32_t k, uint32_t r, uint32_t stride, uint8_t* src,
                                   uint16_t* src_len, const uint8_t* src_mask, const uint8_t* rep,
                                   const uint16_t* rep_size, const uint16_t* rep_len,
                                   const uint8_t* rep_mask, uint32_t sid_base, uint32_t rid_base,
                                   or_decode_status* st, int use_simd)
{
  (void)use_simd;
  gf_init();
  dec_core d;
  gen_sink sink = {src, stride, sid_base, k, src_len};
  core_init(&d, 0, gen_deliver, &sink);
  uint16_t max_len = 0;
  uint32_t m = 0;
  for (uint32_t i = 0; i < k; ++i) {
    if (src_mask[i]) { if (src_len[i] > max_len) max_len = src_len[i]; }
    else ++m;
  }
  memset(st, 0, sizeof *st);
  st->nb_missing = (uint16_t)m;
  /* sources first, ascending id */
  for (uint32_t i = 0; i < k; ++i)
    if (src_mask[i]) core_add_source(&d, sid_base + i, src + (size_t)i * stride, src_len[i]);
  uint32_t* ids = malloc(k * 4);
  for (uint32_t i = 0; i < k; ++i) ids[i] = sid_base + i;
  uint32_t nrecv = 0;
  st->last_repair = 0xFFFF;
  for (uint32_t j = 0; j < r; ++j) {
    if (!rep_mask[j]) continue;
    ++nrecv;
    const size_t before = d.nb_decoded;
    const uint16_t symsz = rep_len ? rep_len[j] : (uint16_t)stride;
    core_add_repair(&d, rid_base + j, ids, k, rep_size[j], rep + (size_t)j * stride, symsz);
    if (d.nb_decoded != before && st->last_repair == 0xFFFF) st->last_repair = (uint16_t)j;
  }
  free(ids);
  st->nb_decoded = (uint16_t)d.nb_decoded;
  st->nb_failed = (uint8_t)(d.nb_failed > 255 ? 255 : d.nb_failed);
  st->nb_useless = (uint16_t)d.nb_useless;
  if (m == 0) st->state = 1;
  else if (d.nb_decoded == m) st->state = 0;
  else if (d.nb_failed) st->state = 3;
  else st->state = 2;
  core_free(&d);
}

void or_decode_generation(uint32_t k, uint32_t r, uint32_t stride, uint8_t* src, uint16_t* src_len,
                          const uint8_t* src_mask, const uint8_t* rep, const uint16_t* rep_size,
                          const uint16_t* rep_len, const uint8_t* rep_mask, uint32_t sid_base,
                          uint32_t rid_base, or_decode_status* st)
{
  decode_generation_impl(k, r, stride, src, src_len, src_mask, rep, rep_size, rep_len, rep_mask,
                         sid_base, rid_base, st, 0);
}

void or_decode_batch(uint32_t G, uint32_t k, uint32_t r, uint32_t stride, uint8_t* src,
                     uint16_t* src_len, const uint8_t* src_mask, const uint8_t* rep,
                     const uint16_t* rep_size, const uint16_t* rep_len, const uint8_t* rep_mask,
                     const uint32_t* sid_base, const uint32_t* rid_base, or_decode_status* st,
                     int use_simd, int nthreads)
{
  gf_init();
  batch_job j;
  memset(&j, 0, sizeof j);
  j.kind = 1; j.k = k; j.r = r; j.stride = stride; j.src = src; j.src_len = src_len;
  j.src_mask = src_mask; j.crep = rep; j.crep_size = rep_size; j.rep_len = rep_len;
  j.rep_mask = rep_mask; j.sid_base = sid_base; j.rid_base = rid_base; j.st = st;
  j.use_simd = use_simd;
  run_batch(&j, G, nthreads);
}

/* ================================================================ wire format ============ */
/* detail/packetizer.hh: big-endian; ids RLE-coded as [count u16][first u32]{[run u8][delta u16]} */

typedef struct { uint8_t* v; size_t n, cap; } bytes;
static void b_put(bytes* b, const void* p, size_t n)
{
  if (b->n + n > b->cap) {
    b->cap = (b->n + n) * 2 + 64;
    b->v = realloc(b->v, b->cap);
  }
  memcpy(b->v + b->n, p, n);
  b->n += n;
}
static void b_u8(bytes* b, uint8_t x) { b_put(b, &x, 1); }
static void b_u16(bytes* b, uint16_t x) { uint8_t t[2] = {(uint8_t)(x >> 8), (uint8_t)x}; b_put(b, t, 2); }
static void b_u32(bytes* b, uint32_t x)
{
  uint8_t t[4] = {(uint8_t)(x >> 24), (uint8_t)(x >> 16), (uint8_t)(x >> 8), (uint8_t)x};
  b_put(b, t, 4);
}

/* packetizer.hh:263-309 */
static void write_ids(bytes* b, const uint32_t* ids, size_t n)
{
  if (n == 0) { b_u16(b, 0); return; }
  uint32_t* diff = malloc(n * 4);
  diff[0] = ids[0];
  for (size_t i = 1; i < n; ++i) diff[i] = ids[i] - ids[i - 1];
  uint8_t* runs = malloc(n);
  uint16_t* vals = malloc(n * 2);
  size_t np = 0;
  size_t c = 1;
  while (c < n) {
    uint8_t run = 1;
    while (c + 1 < n && diff[c] == diff[c + 1] && run < 255) { ++run; ++c; }
    runs[np] = run;
    vals[np] = (uint16_t)diff[c];
    ++np;
    ++c;
  }
  b_u16(b, (uint16_t)(np + 1));
  b_u32(b, ids[0]);
  for (size_t i = 0; i < np; ++i) { b_u8(b, runs[i]); b_u16(b, vals[i]); }
  free(diff); free(runs); free(vals);
}

typedef struct { const uint8_t* p; size_t left; int err; } reader;
static uint8_t r_u8(reader* r)
{
  if (r->left < 1) { r->err = 1; return 0; }
  uint8_t x = r->p[0]; r->p += 1; r->left -= 1; return x;
}
static uint16_t r_u16(reader* r)
{
  if (r->left < 2) { r->err = 1; return 0; }
  uint16_t x = (uint16_t)((r->p[0] << 8) | r->p[1]); r->p += 2; r->left -= 2; return x;
}
static uint32_t r_u32(reader* r)
{
  if (r->left < 4) { r->err = 1; return 0; }
  uint32_t x = ((uint32_t)r->p[0] << 24) | ((uint32_t)r->p[1] << 16) | ((uint32_t)r->p[2] << 8)
             | r->p[3];
  r->p += 4; r->left -= 4; return x;
}

/* packetizer.hh:312-352; result is a sorted unique set (flat_set inserter). */
static void read_ids(reader* r, u32set* out)
{
  memset(out, 0, sizeof *out);
  const uint16_t ne = r_u16(r);
  if (r->err || ne == 0) return;
  uint32_t acc = r_u32(r);
  if (r->err) return;
  u32set_insert(out, acc);
  for (uint32_t i = 0; i + 1 < ne; ++i) {
    const uint8_t run = r_u8(r);
    const uint16_t v = r_u16(r);
    if (r->err) return;
    for (uint32_t j = 0; j < run; ++j) { acc += v; u32set_insert(out, acc); }
  }
}

/* ==================================================== wire format, packet by packet ====== */

/* packetizer.hh:90-122 write_repair: type 1, id, symbol size, symbol, source ids, encoded size,
   symbol size again, symbol again (all integers big-endian).  Returns the packet length. */
size_t or_write_repair_packet(uint32_t rid, const uint8_t* sym, uint16_t symsz, const uint32_t* ids,
                              size_t n, uint16_t esz, uint8_t* out)
{
  bytes b = {0};
  b_u8(&b, 1);
  b_u32(&b, rid);
  b_u16(&b, symsz);
  b_put(&b, sym, symsz);
  write_ids(&b, ids, n);
  b_u16(&b, esz);
  b_u16(&b, symsz);
  b_put(&b, sym, symsz);
  memcpy(out, b.v, b.n);
  const size_t len = b.n;
  free(b.v);
  return len;
}

/* packetizer.hh:165-183 write_source: type 2, id, size, payload. */
size_t or_write_source_packet(uint32_t sid, const uint8_t* data, uint16_t len, uint8_t* out)
{
  bytes b = {0};
  b_u8(&b, 2); b_u32(&b, sid); b_u16(&b, len); b_put(&b, data, len);
  memcpy(out, b.v, b.n);
  const size_t n = b.n;
  free(b.v);
  return n;
}

/* packetizer.hh:46-61 write_ack: type 0, packets received since the last ack, source ids. */
size_t or_write_ack_packet(uint16_t nb_packets, const uint32_t* ids, size_t n, uint8_t* out)
{
  bytes b = {0};
  b_u8(&b, 0); b_u16(&b, nb_packets); write_ids(&b, ids, n);
  memcpy(out, b.v, b.n);
  const size_t len = b.n;
  free(b.v);
  return len;
}

size_t or_packet_bound(size_t symsz, size_t nids) { return 15 + 2 * symsz + 4 + 3 * nids; }

/* packet_type.hh get_packet_type (byte 0) + packetizer.hh:64-88 read_ack, :125-163 read_repair,
 * :186-218 read_source.  Returns the bytes read (the second member of the reference's pair), -1
 * for a packet of unknown type (packet_type_error), -2 for a truncated one (overflow_error). */
long or_parse_packet(const uint8_t* pkt, size_t len, or_packet_view* out)
{
  memset(out, 0, sizeof *out);
  if (len == 0) return -1;
  reader r = {pkt, len, 0};
  const uint8_t ty = r_u8(&r);
  if (ty > 2) return -1;
  out->type = ty;
  u32set ids = {0};
  if (ty == 0) {
    out->nb_packets = r_u16(&r);
    if (r.err) return -2;
    read_ids(&r, &ids);
  } else {
    out->id = r_u32(&r);
    out->symbol_size = r_u16(&r);
    if (r.err || r.left < out->symbol_size) return -2;
    out->symbol_offset = len - r.left;
    r.p += out->symbol_size; r.left -= out->symbol_size;
    if (ty == 1) {
      read_ids(&r, &ids);
      out->encoded_size = r_u16(&r);
    }
  }
  if (r.err) { u32set_free(&ids); return -2; }
  out->ids = ids.v; out->nids = ids.n;
  return (long)(len - r.left);
}

void or_packet_view_free(or_packet_view* v) { free(v->ids); v->ids = NULL; v->nids = 0; }

/* One received packet into a batch's generation layout: the device ingestion's specification
   (ntc_gf256_read_packets, include/netcode/gpu.h).  Parsing follows packetizer.hh:125-158
   (read_repair: the first symbol copy, ids, encoded size; overflow_error on truncation) and
   :186-218 (read_source); get_packet_type (packet.hh) dispatches on byte 0.  Source id s lands in
   generation (s - sid0) / k, slot (s - sid0) % k; repair id likewise with rid0 and r.  A repair is
   stored only if its id list is exactly its generation's k consecutive source ids.  Slots are
   zero-padded to `stride`.  Returns the status code (NTC_PKT_* in gpu.h). */
int or_read_packet_into(const uint8_t* pkt, size_t len, uint32_t G, uint32_t k, uint32_t r,
                        uint32_t stride, uint32_t sid0, uint32_t rid0, uint8_t* src,
                        uint16_t* src_len, uint8_t* src_mask, uint8_t* rep, uint16_t* rep_size,
                        uint8_t* rep_mask)
{
  if (len == 0) return 4;
  reader rd = {pkt, len, 0};
  const uint8_t ty = r_u8(&rd);
  if (ty == 0) return 2;
  if (ty != 1 && ty != 2) return 3;
  const uint32_t id = r_u32(&rd);
  const uint16_t symsz = r_u16(&rd);
  if (rd.err || rd.left < symsz) return 4;
  const uint8_t* sym = rd.p;
  rd.p += symsz; rd.left -= symsz;
  if (ty == 2) {
    const uint32_t d = id - sid0;
    if ((uint64_t)d >= (uint64_t)G * k) return 5;
    if (symsz > stride) return 6;
    uint8_t* dst = src + (size_t)d * stride;
    memcpy(dst, sym, symsz);
    memset(dst + symsz, 0, stride - symsz);
    src_len[d] = symsz;
    src_mask[d] = 1;
    return 0;
  }
  u32set ids;
  read_ids(&rd, &ids);
  const uint16_t esz = r_u16(&rd);
  if (rd.err) { u32set_free(&ids); return 4; }
  const uint32_t d = id - rid0;
  if ((uint64_t)d >= (uint64_t)G * r) { u32set_free(&ids); return 5; }
  if (symsz > stride) { u32set_free(&ids); return 6; }
  const uint32_t g = d / r, sidb = sid0 + g * k;
  int full = ids.n == k;
  for (size_t i = 0; full && i < ids.n; ++i) full = ids.v[i] == sidb + (uint32_t)i;
  u32set_free(&ids);
  if (!full) return 7;
  uint8_t* dst = rep + (size_t)d * stride;
  memcpy(dst, sym, symsz);
  memset(dst + symsz, 0, stride - symsz);
  rep_size[d] = esz;
  rep_mask[d] = 1;
  return 1;
}

/* ======================================================== public encoder (encoder.hh) ====== */
typedef struct { uint32_t id; uint16_t len; uint8_t* data; } esrc;

struct or_encoder {
  int w;                                   /* Galois field size (galois_field.hh:35-44) */
  int systematic, adaptive;
  size_t rate, window_size;
  uint32_t cur_sid, cur_rid;
  esrc* win; size_t nwin, capwin;          /* insertion (= id) order */
  size_t nb_repairs, nb_acks, nb_sources;
  uint16_t nb_sent_packets;
  or_emit_fn emit; void* ctx;
};

or_encoder* or_encoder_new(or_emit_fn emit, void* ctx)
{
  gf_init();
  or_encoder* e = calloc(1, sizeof *e);
  e->w = 8;
  e->systematic = 1; e->rate = 5; e->window_size = (size_t)-1;
  e->emit = emit; e->ctx = ctx;
  return e;
}
void or_encoder_free(or_encoder* e)
{
  for (size_t i = 0; i < e->nwin; ++i) free(e->win[i].data);
  free(e->win); free(e);
}
void or_encoder_set_rate(or_encoder* e, size_t r) { e->rate = r; }
void or_encoder_set_window_size(or_encoder* e, size_t s) { e->window_size = s; }
void or_encoder_set_code_type(or_encoder* e, int s) { e->systematic = s; }
void or_encoder_set_adaptive(or_encoder* e, int a) { e->adaptive = a; }
size_t or_encoder_window(const or_encoder* e) { return e->nwin; }
size_t or_encoder_rate(const or_encoder* e) { return e->rate; }
size_t or_encoder_nb_sent_repairs(const or_encoder* e) { return e->nb_repairs; }
size_t or_encoder_nb_sent_sources(const or_encoder* e) { return e->nb_sources; }
size_t or_encoder_nb_received_acks(const or_encoder* e) { return e->nb_acks; }

/* detail/encoder.cc:15-64 in the calling thread's field: sym[0..max len) = sum_i c(rid, ids[i]) *
 * syms[i] (each zero-extended), *esz = XOR of the coded lengths.  Returns the symbol length. */
static uint16_t build_repair(uint32_t rid, size_t n, const uint32_t* ids, const uint8_t* const* syms,
                             const uint16_t* lens, uint8_t* sym, uint16_t* esz)
{
  uint16_t symsz = 0;
  for (size_t i = 0; i < n; ++i) if (lens[i] > symsz) symsz = lens[i];
  memset(sym, 0, symsz);
  uint16_t e = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint32_t c = or_coefficient(rid, ids[i]);
    if (i == 0) or_region_mul(syms[i], sym, lens[i], c);        /* :26-35 the first source */
    else or_region_muladd(syms[i], sym, lens[i], c);            /* :38-62 the others */
    e = (uint16_t)(or_multiply_size(lens[i], c) ^ e);
  }
  *esz = e;
  return symsz;
}

uint16_t or_build_repair(int w, uint32_t rid, size_t n, const uint32_t* ids, const uint8_t* const* syms,
                         const uint16_t* lens, uint8_t* sym, uint16_t* esz)
{
  gf_init();
  const int old = g_w; g_w = w;
  const uint16_t r = build_repair(rid, n, ids, syms, lens, sym, esz);
  g_w = old;
  return r;
}

/* encoder.hh:162-169, 321-333 + packetizer.hh:90-122 */
static void enc_generate_repair(or_encoder* e)
{
  uint16_t symsz = 0;
  for (size_t i = 0; i < e->nwin; ++i) if (e->win[i].len > symsz) symsz = e->win[i].len;
  uint8_t* sym = calloc((size_t)symsz + 16, 1);
  uint16_t esz = 0;
  uint32_t* ids = malloc((e->nwin + 1) * 4);
  const uint8_t** syms = malloc((e->nwin + 1) * sizeof(void*));
  uint16_t* lens = malloc((e->nwin + 1) * 2);
  for (size_t i = 0; i < e->nwin; ++i) { ids[i] = e->win[i].id; syms[i] = e->win[i].data; lens[i] = e->win[i].len; }
  build_repair(e->cur_rid, e->nwin, ids, syms, lens, sym, &esz);
  free(syms); free(lens);
  /* source_ids is a flat_set: ids inserted in window order are ascending */
  bytes b = {0};
  b_u8(&b, 1);
  b_u32(&b, e->cur_rid);
  b_u16(&b, symsz);
  b_put(&b, sym, symsz);
  write_ids(&b, ids, e->nwin);
  b_u16(&b, esz);
  b_u16(&b, symsz);
  b_put(&b, sym, symsz);
  e->cur_rid++;
  e->nb_repairs++;
  e->nb_sent_packets++;
  e->emit(e->ctx, b.v, b.n);
  free(b.v); free(sym); free(ids);
}

/* encoder.hh:255-285 */
static void enc_add_data(or_encoder* e, const uint8_t* data, uint16_t len)
{
  if (e->nwin == e->window_size) {
    free(e->win[0].data);
    memmove(e->win, e->win + 1, (e->nwin - 1) * sizeof(esrc));
    e->nwin--;
  }
  if (e->nwin == e->capwin) {
    e->capwin = e->capwin ? 2 * e->capwin : 64;
    e->win = realloc(e->win, e->capwin * sizeof(esrc));
  }
  esrc* s = &e->win[e->nwin++];
  s->id = e->cur_sid; s->len = len;
  s->data = malloc((size_t)len + 16);
  memcpy(s->data, data, len);
  if (e->systematic) {
    e->nb_sources++;
    e->nb_sent_packets++;
    bytes b = {0};                                    /* packetizer.hh:165-183 */
    b_u8(&b, 2); b_u32(&b, s->id); b_u16(&b, len); b_put(&b, data, len);
    e->emit(e->ctx, b.v, b.n);
    free(b.v);
  } else {
    enc_generate_repair(e);
  }
  if ((e->cur_sid + 1) % e->rate == 0) enc_generate_repair(e);
  e->cur_sid++;
}

/* encoder.hh:290-318 + packetizer.hh:64-88 + source_list.hh:34-60 */
long or_encoder_add_packet(or_encoder* e, const uint8_t* pkt, size_t len)
{
  if (len == 0 || pkt[0] != 0) return -1;
  e->nb_acks++;
  or_packet_view v;
  const long consumed = or_parse_packet(pkt, len, &v);
  if (consumed < 0) return consumed;
  const uint16_t nbp = v.nb_packets;
  u32set ids = {v.ids, v.nids, v.nids};
  if (e->adaptive) {
    double loss = 0.0;
    if (e->nb_sent_packets > 0)
      loss = (double)(e->nb_sent_packets - nbp) / (double)e->nb_sent_packets;
    if (loss < 0.01) e->rate = 50;
    else { double q = (1.0 / loss) / 2.0; size_t c = (size_t)q; if ((double)c < q) c++; e->rate = c; }
  }
  e->nb_sent_packets = 0;
  size_t si = 0, ii = 0;
  while (si < e->nwin && ii < ids.n) {
    if (e->win[si].id == ids.v[ii]) {
      free(e->win[si].data);
      memmove(e->win + si, e->win + si + 1, (e->nwin - si - 1) * sizeof(esrc));
      e->nwin--;
      ++ii;
    } else if (e->win[si].id > ids.v[ii]) {
      ++ii;
    } else {
      ++si;
    }
  }
  u32set_free(&ids);
  return consumed;
}

/* ======================================================== public decoder (decoder.hh) ====== */
struct or_decoder {
  int w;
  dec_core core;
  uint16_t ack_nb_packets;
  long ack_period_ms;
  struct timespec last_ack;
  uint16_t ack_packets;
  size_t nb_rrep, nb_rsrc, nb_acks;
  or_emit_fn emit; void* ectx;
  or_deliver_fn deliver; void* dctx;
};

static double ts_ms(struct timespec a) { return a.tv_sec * 1e3 + a.tv_nsec / 1e6; }

/* decoder.hh:213-228 */
void or_decoder_generate_ack(or_decoder* d)
{
  bytes b = {0};
  b_u8(&b, 0);
  b_u16(&b, d->ack_packets);
  uint32_t* ids = malloc((d->core.nsrc + 1) * 4);
  for (size_t i = 0; i < d->core.nsrc; ++i) ids[i] = d->core.src[i].id;
  write_ids(&b, ids, d->core.nsrc);
  free(ids);
  d->nb_acks++;
  d->ack_packets = 0;
  d->emit(d->ectx, b.v, b.n);
  free(b.v);
}

/* decoder.hh:231-248 */
void or_decoder_maybe_ack(or_decoder* d)
{
  if (d->ack_packets >= d->ack_nb_packets) {
    or_decoder_generate_ack(d);
    clock_gettime(CLOCK_MONOTONIC, &d->last_ack);
  } else if (d->ack_period_ms != 0) {
    struct timespec now;
    clock_gettime(CLOCK_MONOTONIC, &now);
    if (ts_ms(now) - ts_ms(d->last_ack) >= (double)d->ack_period_ms) {
      or_decoder_generate_ack(d);
      d->last_ack = now;
    }
  }
}

/* decoder.hh:292-300 */
static void pub_handle_source(void* ctx, const dsrc* s)
{
  or_decoder* d = (or_decoder*)ctx;
  d->deliver(d->dctx, s->id, s->data, s->len);
  or_decoder_maybe_ack(d);
}

or_decoder* or_decoder_new(int in_order, or_emit_fn emit, void* ectx, or_deliver_fn deliver,
                           void* dctx)
{
  gf_init();
  or_decoder* d = calloc(1, sizeof *d);
  d->w = 8;
  core_init(&d->core, in_order, pub_handle_source, d);
  d->ack_nb_packets = 50;
  d->ack_period_ms = 100;
  clock_gettime(CLOCK_MONOTONIC, &d->last_ack);
  d->emit = emit; d->ectx = ectx; d->deliver = deliver; d->dctx = dctx;
  return d;
}
void or_decoder_free(or_decoder* d) { core_free(&d->core); free(d); }
void or_decoder_set_ack_nb_packets(or_decoder* d, uint16_t nb) { d->ack_nb_packets = nb < 128 ? nb : 128; }
void or_decoder_set_ack_period_ms(or_decoder* d, long ms) { d->ack_period_ms = ms; }

size_t or_decoder_counter(const or_decoder* d, int which)
{
  switch (which) {
    case 0: return d->core.nb_decoded;
    case 1: return d->core.nb_failed;
    case 2: return d->core.nmiss;
    case 3: return d->nb_rrep;
    case 4: return d->nb_rsrc;
    case 5: return d->nb_acks;
    case 6: return d->core.nb_useless;
    case 7: return d->core.nrep;
    default: return 0;
  }
}

/* decoder.hh:88-122 + packetizer.hh:125-218 */
static long dec_add_packet(or_decoder* d, const uint8_t* pkt, size_t len)
{
  if (len == 0 || (pkt[0] != 1 && pkt[0] != 2)) return -1;     /* decoder.hh:117-120 */
  if (pkt[0] == 1) d->nb_rrep++;                                 /* counted before parsing */
  else d->nb_rsrc++;
  d->ack_packets++;
  or_packet_view v;
  const long consumed = or_parse_packet(pkt, len, &v);
  if (consumed < 0) return consumed;
  if (v.type == 1) {
    if (v.nids) core_add_repair(&d->core, v.id, v.ids, v.nids, v.encoded_size, pkt + v.symbol_offset,
                                v.symbol_size);
  } else {
    core_add_source(&d->core, v.id, pkt + v.symbol_offset, v.symbol_size);
  }
  or_packet_view_free(&v);
  return consumed;
}

/* ============================================================= loss models =============== */
/* libstdc++ minstd_rand0: x = 16807 x mod (2^31-1), default seed 1. */
static uint32_t minstd_next(uint32_t* s)
{
  *s = (uint32_t)(((uint64_t)*s * 16807u) % 2147483647u);
  return *s;
}
/* libstdc++ uniform_int_distribution<unsigned>{1,100} over minstd_rand0 (downscaling path). */
static unsigned uid_1_100(uint32_t* s)
{
  const uint64_t urngrange = 2147483646u - 1u;  /* max - min */
  const uint64_t urange = 99;
  const uint64_t uerange = urange + 1;
  const uint64_t scaling = urngrange / uerange;
  const uint64_t past = uerange * scaling;
  uint64_t ret;
  do { ret = (uint64_t)minstd_next(s) - 1u; } while (ret >= past);
  return (unsigned)(ret / scaling) + 1u;
}
void or_burst_init(or_burst* b, unsigned good, unsigned bad)
{
  b->state = 1; b->bad = 0; b->good_th = good; b->bad_th = bad;
}
/* tools/loss/burst.hh:27-58 */
int or_burst_next(or_burst* b)
{
  if (!b->bad) {
    if (uid_1_100(&b->state) < b->good_th) return 0;
    b->bad = 1; return 1;
  }
  if (uid_1_100(&b->state) < b->bad_th) return 1;
  b->bad = 0; return 0;
}
void or_uniform_init(or_uniform* u, unsigned threshold) { u->state = 1; u->threshold = threshold; }
int or_uniform_next(or_uniform* u) { return uid_1_100(&u->state) > u->threshold; }  /* uniform.hh:26-28 */

/* ============================================================ end_to_end harness ========= */
typedef struct { bytes* pk; size_t n, cap; } pktq;
static void q_emit(void* ctx, const uint8_t* p, size_t n)
{
  pktq* q = (pktq*)ctx;
  if (q->n == q->cap) { q->cap = q->cap ? 2 * q->cap : 16; q->pk = realloc(q->pk, q->cap * sizeof(bytes)); }
  q->pk[q->n].v = malloc(n ? n : 1);
  memcpy(q->pk[q->n].v, p, n);
  q->pk[q->n].n = n; q->pk[q->n].cap = n;
  q->n++;
}
static void q_clear(pktq* q) { for (size_t i = 0; i < q->n; ++i) free(q->pk[i].v); q->n = 0; }

typedef struct { uint64_t nb; uint32_t expected; uint16_t psz; int bad; } e2e_sink;
static void e2e_deliver(void* ctx, uint32_t id, const uint8_t* data, size_t len)
{
  (void)id;
  e2e_sink* s = (e2e_sink*)ctx;                      /* end_to_end.cc:50-73 */
  if (len != s->psz) { s->bad = 1; return; }
  uint32_t first; memcpy(&first, data, 4);
  if (first != s->expected) { s->bad = 1; return; }
  for (size_t i = 0; i < len / 4; ++i) {
    uint32_t w; memcpy(&w, data + 4 * i, 4);
    if (w != first) { s->bad = 1; return; }
  }
  s->nb++;
  s->expected++;
}

/* Public entry points that do field arithmetic run in the object's field. */
void or_encoder_generate_repair(or_encoder* e)
{
  const int old = g_w; g_w = e->w; enc_generate_repair(e); g_w = old;
}
void or_encoder_add_data(or_encoder* e, const uint8_t* data, uint16_t len)
{
  const int old = g_w; g_w = e->w; enc_add_data(e, data, len); g_w = old;
}
long or_decoder_add_packet(or_decoder* d, const uint8_t* pkt, size_t len)
{
  const int old = g_w; g_w = d->w; const long n = dec_add_packet(d, pkt, len); g_w = old;
  return n;
}
void or_encoder_set_field(or_encoder* e, int w) { e->w = w; }
void or_decoder_set_field(or_decoder* d, int w) { d->w = w; }

int or_end_to_end(uint32_t nb_packets, uint64_t* out)
{
  const uint16_t psz = 1024;
  or_burst loss; or_burst_init(&loss, 95, 5);
  pktq eq = {0}, dq = {0};
  e2e_sink sink = {0, 0, psz, 0};
  or_encoder* enc = or_encoder_new(q_emit, &eq);
  or_decoder* dec = or_decoder_new(1, q_emit, &dq, e2e_deliver, &sink);
  or_decoder_set_ack_period_ms(dec, 0);
  uint64_t to_dec_loss = 0;
  uint32_t id = 0;
  uint8_t* data = malloc(psz);
  while (id < nb_packets) {
    for (uint32_t w = 0; w < psz / 4; ++w) memcpy(data + 4 * w, &id, 4);
    id++;
    or_encoder_add_data(enc, data, psz);
    for (size_t i = 0; i < eq.n; ++i) {
      if (!or_burst_next(&loss)) or_decoder_add_packet(dec, eq.pk[i].v, eq.pk[i].n);
      else ++to_dec_loss;
    }
    if (((dec->nb_rsrc + dec->nb_rrep) % 50) == 0) {
      or_decoder_generate_ack(dec);
      for (size_t i = 0; i < dq.n; ++i)
        if (!or_burst_next(&loss)) or_encoder_add_packet(enc, dq.pk[i].v, dq.pk[i].n);
    }
    q_clear(&eq);
    q_clear(&dq);
  }
  out[0] = id; out[1] = to_dec_loss; out[2] = dec->nb_rrep; out[3] = dec->nb_rsrc;
  out[4] = dec->core.nb_useless; out[5] = dec->core.nb_decoded; out[6] = sink.nb;
  const int bad = sink.bad;
  free(data);
  free(eq.pk); free(dq.pk);
  or_encoder_free(enc);
  or_decoder_free(dec);
  return bad ? -1 : 0;
}

/* ================================================ per-packet workload (CPU baseline leg) ==== */
/* bench.py --per-packet, C level: F flows x M items of S bytes through one ntc::encoder per flow
 * (window W, a repair every R sources), then each flow's packets with an i.i.d. loss of L % fed to
 * its own in-order decoder, round-robin over flows -- the reference's usage, one call per packet.
 * The GPU side (tools/pp_driver.c over libntc.so) draws the same payloads and losses, so both
 * produce the same packets and deliveries (hashes compared).  Timed: the encode calls, the decode
 * calls.  secs[0..1] = encode, decode; counts[0..3] = packets, received packets, deliveries,
 * repairs; hashes[0..1] = FNV-1a over every flow's packets, over every flow's deliveries. */
static uint64_t pp_mix(uint64_t x)
{
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static uint64_t pp_fnv(uint64_t h, const uint8_t* p, size_t n)
{
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return h;
}

typedef struct { uint8_t* v; size_t n, cap; size_t* off; size_t np, capp; } pp_store;

static void pp_push(pp_store* s, const uint8_t* p, size_t n)
{
  if (s->n + n > s->cap) {
    s->cap = (s->n + n) * 2 + 4096;
    s->v = (uint8_t*)realloc(s->v, s->cap);
  }
  if (s->np + 2 > s->capp) {
    s->capp = s->capp * 2 + 64;
    s->off = (size_t*)realloc(s->off, s->capp * sizeof(size_t));
  }
  if (s->np == 0) s->off[0] = 0;
  memcpy(s->v + s->n, p, n);
  s->n += n;
  s->off[++s->np] = s->n;
}

/* the application's stores are sized and paged in before the clock starts (tools/pp_driver.c does
 * the same) */
static void pp_reserve(pp_store* s, size_t bytes, size_t items)
{
  s->cap = bytes;
  s->v = (uint8_t*)malloc(bytes);
  memset(s->v, 0, bytes);
  s->capp = items + 2;
  s->off = (size_t*)malloc(s->capp * sizeof(size_t));
}

static void pp_emit(void* ctx, const uint8_t* p, size_t n) { pp_push((pp_store*)ctx, p, n); }
static void pp_deliver(void* ctx, uint32_t id, const uint8_t* p, size_t n)
{
  (void)id;
  pp_push((pp_store*)ctx, p, n);
}

static double pp_now(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int or_pp_bench(uint32_t F, uint32_t M, uint32_t S, uint32_t W, uint32_t R, uint32_t loss_pct,
                uint64_t seed, double* secs, uint64_t* counts, uint64_t* hashes)
{
  gf_init();
  uint8_t* data = (uint8_t*)malloc((size_t)M * S + 8);
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t b = 0; b < S; ++b)
      data[(size_t)i * S + b] = (uint8_t)(pp_mix(seed + ((uint64_t)i << 32) + b / 8) >> (8 * (b % 8)));
  pp_store* tx = (pp_store*)calloc(F, sizeof(pp_store));
  pp_store* rx = (pp_store*)calloc(F, sizeof(pp_store));
  pp_store* acks = (pp_store*)calloc(F, sizeof(pp_store));
  or_encoder** enc = (or_encoder**)calloc(F, sizeof(or_encoder*));
  or_decoder** dec = (or_decoder**)calloc(F, sizeof(or_decoder*));
  for (uint32_t f = 0; f < F; ++f) {
    pp_reserve(&tx[f], (size_t)M * (S + 16) + (size_t)((R ? M / R : M) + 1) * (2 * S + 256), 2 * (size_t)M + 64);
    pp_reserve(&rx[f], (size_t)M * S + 4096, (size_t)M + 64);
    enc[f] = or_encoder_new(pp_emit, &tx[f]);
    or_encoder_set_rate(enc[f], R);
    or_encoder_set_window_size(enc[f], W);
  }
  double t0 = pp_now();
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t f = 0; f < F; ++f) or_encoder_add_data(enc[f], data + (size_t)i * S, (uint16_t)S);
  secs[0] = pp_now() - t0;
  uint64_t npk = 0, nrep = 0, nrx = 0, ndel = 0;
  for (uint32_t f = 0; f < F; ++f) { npk += tx[f].np; nrep += or_encoder_nb_sent_repairs(enc[f]); }
  /* the received streams: packet j of flow f survives iff mix(seed, f, j) % 100 >= loss_pct */
  uint32_t** keep = (uint32_t**)calloc(F, sizeof(uint32_t*));
  uint32_t* nkeep = (uint32_t*)calloc(F, sizeof(uint32_t));
  uint32_t rounds = 0;
  for (uint32_t f = 0; f < F; ++f) {
    keep[f] = (uint32_t*)malloc((tx[f].np + 1) * sizeof(uint32_t));
    for (uint32_t j = 0; j < tx[f].np; ++j)
      if (pp_mix(seed ^ 0x5EEDull ^ ((uint64_t)f << 40) ^ j) % 100 >= loss_pct) keep[f][nkeep[f]++] = j;
    nrx += nkeep[f];
    if (nkeep[f] > rounds) rounds = nkeep[f];
    dec[f] = or_decoder_new(1, pp_emit, &acks[f], pp_deliver, &rx[f]);
    or_decoder_set_ack_period_ms(dec[f], 0);
  }
  t0 = pp_now();
  for (uint32_t i = 0; i < rounds; ++i)
    for (uint32_t f = 0; f < F; ++f)
      if (i < nkeep[f]) {
        const uint32_t j = keep[f][i];
        or_decoder_add_packet(dec[f], tx[f].v + tx[f].off[j], tx[f].off[j + 1] - tx[f].off[j]);
      }
  secs[1] = pp_now() - t0;
  uint64_t hp = 0xCBF29CE484222325ull, hd = 0xCBF29CE484222325ull;
  for (uint32_t f = 0; f < F; ++f) {
    hp = pp_fnv(hp, tx[f].v, tx[f].n);
    hd = pp_fnv(hd, rx[f].v, rx[f].n);
    ndel += rx[f].np;
  }
  counts[0] = npk; counts[1] = nrx; counts[2] = ndel; counts[3] = nrep;
  hashes[0] = hp; hashes[1] = hd;
  for (uint32_t f = 0; f < F; ++f) {
    or_encoder_free(enc[f]);
    or_decoder_free(dec[f]);
    free(tx[f].v); free(tx[f].off); free(rx[f].v); free(rx[f].off);
    free(acks[f].v); free(acks[f].off); free(keep[f]);
  }
  free(tx); free(rx); free(acks); free(enc); free(dec); free(keep); free(nkeep); free(data);
  return 0;
}
