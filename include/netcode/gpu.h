/*
 * netcode/gpu.h -- batched GF(2^8) network-coding engine for MI355X (gfx950).
 *
 * C ABI (plain pointers and sizes, no HIP/torch types) behind which the hand-written CDNA4 HIP
 * kernels of libntc_gf256.so run.  It replaces, for whole batches of independent generations,
 * the reference's per-packet GF region calls:
 *
 *   ntc_gf256_encode_batch   <- ntc::detail::encoder::operator()   netcode/detail/encoder.cc:15-64
 *                               (galois_field::multiply / multiply_add / multiply_size,
 *                                netcode/detail/galois_field.hh:65-120), one call per repair in
 *                               ntc::encoder::generate_repair (netcode/encoder.hh:162-169).
 *   ntc_gf256_decode_batch   <- ntc::detail::decoder::operator()(decoder_repair&&) and
 *                               attempt_full_decoding (netcode/detail/decoder.cc:54-152,
 *                               393-408, 412-566) + detail::invert (invert_matrix.cc:9-128).
 *   ntc_gf256_region_multiply<- galois_field::multiply / multiply_add (galois_field.hh:65-92).
 *   ntc_gf256_coefficient    <- galois_field::coefficient (galois_field.hh:143-158, w = 8).
 *   ntc_gf256_multiply_size  <- galois_field::multiply_size (galois_field.hh:96-120, w = 8).
 *
 * Layout contract (all device pointers, caller-owned, HBM-resident):
 *   src       [G][k][stride] bytes, slot i of generation g holds source id sid_base[g] + i,
 *             zero-padded after src_len[g][i] bytes (the reference zero-pads shorter sources,
 *             detail/encoder.cc:44-48).
 *   rep       [G][r][stride] bytes, slot j holds repair id rid_base[g] + j.
 *   stride    multiple of 16, >= the longest symbol; symbols are u16-sized (<= 65535 B).
 *   sid_base / rid_base: [G] u32 or NULL (then g*k and g*r).  Ids must not wrap inside a
 *             generation (sid_base + k <= 2^32); the coefficient product itself wraps exactly
 *             like the reference's uint32 arithmetic.
 * All calls are asynchronous on `stream` (a hipStream_t, NULL = default stream) and return an
 * ntc_gpu_status; no exceptions cross the ABI.  One engine per device; not thread-safe.
 */
#ifndef NETCODE_GPU_H
#define NETCODE_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  NTC_GPU_OK = 0,
  NTC_GPU_EINVAL = 1,        /* bad argument (sizes, alignment, NULL) */
  NTC_GPU_ENOMEM = 2,        /* device workspace allocation failed */
  NTC_GPU_EDEVICE = 3,       /* HIP runtime error (launch / device) */
  NTC_GPU_EUNSUPPORTED = 4   /* shape outside this build's limits (e.g. decode r > 255) */
} ntc_gpu_status;

/* Per-generation decode outcome; the same fields the reference decoder's counters expose
 * (detail/decoder.cc nb_decoded / nb_failed_full_decodings / nb_useless_repairs) when the
 * generation's received sources and then its received repairs are fed in ascending id order. */
typedef struct {
  uint8_t  state;        /* 0 decoded, 1 nothing missing, 2 not enough repairs, 3 all attempts
                            singular (every candidate matrix non-invertible) */
  uint8_t  nb_failed;    /* failed full decodings (singular matrices; detail/decoder.cc:448-468) */
  uint16_t nb_missing;   /* m = lost sources in the generation */
  uint16_t nb_decoded;   /* sources recovered */
  uint16_t nb_useless;   /* repairs dropped as useless (detail/decoder.cc:77-89) */
  uint16_t last_repair;  /* slot of the repair that completed decoding, 0xFFFF if none */
  uint16_t pad;
} ntc_gf256_decode_status;

typedef struct ntc_gf256_engine ntc_gf256_engine;

/* Create an engine bound to HIP device `device`; builds the device-resident coefficient tables. */
int  ntc_gf256_engine_create(int device, ntc_gf256_engine** out);
void ntc_gf256_engine_destroy(ntc_gf256_engine* eng);

/* Region-MAC formulation (tuning and A/B testing; results are identical).  AUTO picks the
 * bit-sliced XOR kernel when the stride fills >= 1/3 of its 2 KiB wave span (stride % 16 == 0),
 * the v_perm kernel otherwise; the NTC_GF256_MAC=perm|bitslice|grouped|paired environment variable
 * overrides AUTO process-wide.  BITSLICE runs one independent wave per row tile (gf_mac_bs);
 * BITSLICE_GROUPED (experimental, slower on MI355X: DESIGN.md §3) runs pairs of 16-row tiles per
 * workgroup that build each source's bit planes once and share them through LDS (gf_mac_bsg);
 * BITSLICE_PAIRED (experimental, 1-3 % slower on MI355X: DESIGN.md §3) runs the two 16-row tiles
 * of a (generation, span) as one 2-wave workgroup in which each wave transposes half the sources
 * and publishes only their 8 planes to the other (gf_mac_bsp; NTC_GF256_MAC=paired, with
 * NTC_GF256_PAIRJ=1|2 sources per wave and turn, NTC_GF256_PAIRSETS=3|4 LDS slot sets).
 * An encode / combine with >= 384 rows over whole 2 KiB spans (BITSLICE or AUTO) first bit-slices
 * its sources into an engine buffer (one HBM pass), so the MAC's row tiles skip the per-tile
 * transpose.  More environment variables, for experiments only (results identical):
 * NTC_GF256_ROWTILE=8|16 fixes the bit-sliced row tile (default: 16 when a tile has more than 8
 * rows), NTC_GF256_KSPLIT=n (1..8) fixes the split-k part count of encodes with too few tasks to
 * fill the GPU, NTC_GF256_SLICE=0|1 turns the source pre-slicing off / on for every eligible call. */
enum { NTC_GF256_MAC_AUTO = 0, NTC_GF256_MAC_PERM = 1, NTC_GF256_MAC_BITSLICE = 2,
       NTC_GF256_MAC_BITSLICE_GROUPED = 3, NTC_GF256_MAC_BITSLICE_PAIRED = 4 };
int  ntc_gf256_set_mac_kind(ntc_gf256_engine* eng, int kind);

/* Decode-plan kernel (coverage and A/B testing; results are identical).  AUTO: the register-
 * resident wave plan for r <= 32, the LDS wave plan for r <= 64, the workgroup plan above; WAVE /
 * LDS fall back to the next kernel when r exceeds their limit (32 / 64); BIG forces the
 * workgroup plan for every r.  The NTC_GF256_PLAN=lds|big environment variable overrides AUTO. */
enum { NTC_GF256_PLAN_AUTO = 0, NTC_GF256_PLAN_WAVE = 1, NTC_GF256_PLAN_LDS = 2,
       NTC_GF256_PLAN_BIG = 3 };
int  ntc_gf256_set_plan_kind(ntc_gf256_engine* eng, int kind);

/* Profiling: with timing on, the engine records HIP events on the caller's stream around each
 * region-MAC kernel launch; ntc_gf256_mac_time waits for the last encode (dec = 0) or decode
 * (dec = 1) MAC and returns that kernel's duration in ms. */
int  ntc_gf256_set_timing(ntc_gf256_engine* eng, int on);
int  ntc_gf256_mac_time(ntc_gf256_engine* eng, int dec, float* ms);

/* Kernel timing log: after ntc_gf256_timing_log(eng, capacity > 0) the engine brackets each of
 * the next `capacity` kernels it launches with a HIP event pair on the launch stream (capacity 0
 * turns the log off; every call clears it).  ntc_gf256_timing_read waits for the logged kernels
 * and returns up to `max` entries in launch order: kinds[i] (NTC_GF256_K_*) and ms[i] (that
 * kernel's duration); *n = entries logged.  bench.py times the kernels of its timed steps this
 * way, so per-step kernel sums come from the same launches as the step time.
 * ntc_gf256_timing_kinds restricts the log to the kinds whose bit (1 << NTC_GF256_K_*) is set in
 * `mask` (default: all): every logged kernel costs two event records on its stream, a few
 * microseconds that matter for sub-millisecond steps. */
enum { NTC_GF256_K_ENCODE_PREP = 0, NTC_GF256_K_ENCODE_MAC = 1, NTC_GF256_K_DECODE_PLAN = 2,
       NTC_GF256_K_PLAN_ROWS = 3, NTC_GF256_K_DECODE_MAC = 4, NTC_GF256_K_BJ_OFFSETS = 5 /* reserved */,
       NTC_GF256_K_DENSE = 6, NTC_GF256_K_OTHER = 7 /* the split-k MAC's part reduction */,
       NTC_GF256_K_SLICE = 8 /* a tall encode / combine's source pre-slicing pass */ };
int  ntc_gf256_timing_log(ntc_gf256_engine* eng, uint32_t capacity);
int  ntc_gf256_timing_kinds(ntc_gf256_engine* eng, uint32_t mask);
int  ntc_gf256_timing_read(ntc_gf256_engine* eng, uint32_t max, uint32_t* n, uint32_t* kinds,
                           float* ms);

/* Pre-size the decode workspace for (G, k, r) so later calls never allocate (graph capture).
 * A bit-sliced encode / combine with fewer tasks than one round of wave slots (few generations,
 * k >= 128) splits its sources (split-k) and sizes its partial outputs on first use; a call
 * captured before that first use runs unsplit instead of allocating (identical results).  The
 * pre-sliced source copy of a tall encode / combine is sized the same way (captured before its
 * first use: the MAC slices in registers instead).  Both are optimisations: when the device has
 * no room for them the call runs without them (identical results) instead of failing.  Once any
 * call of an engine has been captured, a workspace buffer that a later, larger call outgrows is
 * kept (not freed) until the engine is destroyed or ntc_gf256_release_retired is called, so
 * captured graphs never address freed memory; from then on buffers grow at least 2x at a time,
 * so the retired memory stays below the current workspace (split-k parts and the sliced copy are
 * G * k * stride bytes scale: 64 MiB each at k = 1024, 64 KiB, G = 1). */
int  ntc_gf256_reserve(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r);
/* Free the workspace buffers retired after a capture.  Only once no graph captured from this
 * engine will be launched again (e.g. after hipGraphExecDestroy of all of them). */
int  ntc_gf256_release_retired(ntc_gf256_engine* eng);

/* Encode: rep[g][j] = sum_i c(rid_base[g]+j, sid_base[g]+i) * src[g][i] over GF(2^8)/0x11D.
 * Any r (the coefficient walk runs in chunks of 256 rows); k <= 65535.
 * rep_size[g][j] = encoded size (XOR of bytewise-coded u16 lengths); rep_len[g] = repair symbol
 * length = max src_len over the generation (may be NULL). */
int  ntc_gf256_encode_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                            uint32_t stride, const uint8_t* src, const uint16_t* src_len,
                            const uint32_t* sid_base, const uint32_t* rid_base, uint8_t* rep,
                            uint16_t* rep_size, uint16_t* rep_len, void* stream);

/* Decode in place: lost source slots (src_mask == 0) whose generation decodes are overwritten
 * with the recovered payload (zero-padded to stride) and their src_len set to the decoded size.
 * status[g] receives the outcome.  Requires r <= 255 (r <= 64: wave-level plan kernels; 64 < r
 * <= 255: one workgroup per generation, decode_plan_big). */
int  ntc_gf256_decode_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                            uint32_t stride, uint8_t* src, uint16_t* src_len,
                            const uint8_t* src_mask, const uint8_t* rep, const uint16_t* rep_size,
                            const uint8_t* rep_mask, const uint32_t* sid_base,
                            const uint32_t* rid_base, ntc_gf256_decode_status* status,
                            void* stream);

/* The two halves of ntc_gf256_decode_batch, exposed for profiling: the per-generation plan
 * (greedy repair selection + device Gauss-Jordan, writes status and decoded sizes) and the
 * region multiply-accumulate that applies it. */
int  ntc_gf256_decode_plan(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                           uint16_t* src_len, const uint8_t* src_mask, const uint16_t* rep_size,
                           const uint8_t* rep_mask, const uint32_t* sid_base,
                           const uint32_t* rid_base, ntc_gf256_decode_status* status,
                           void* stream);
int  ntc_gf256_decode_apply(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                            uint32_t stride, uint8_t* src, const uint8_t* rep, void* stream);

/* General batched combination with caller-supplied coefficients (no id schedule):
 *   out[g][j] = sum_i coef[g][i][j] * in[g][i]      (j < rows, i < k), over `stride` bytes,
 * coef laid out [G][k][ntc_gf256_coef_pitch(rows)] bytes (entries j >= rows ignored).  Used by
 * the per-packet netcode/c layer (one repair or one decoded source = one row) and by dense
 * non-reference codes (BASELINE config 5). */
uint32_t ntc_gf256_coef_pitch(uint32_t rows);
int  ntc_gf256_combine_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t rows,
                             uint32_t stride, const uint8_t* in, const uint8_t* coef,
                             uint8_t* out, void* stream);

/* Gathered combination over payloads that already live on the device (the per-packet batching
 * adaptor's resident payload arena, netcode/c/ext.h ntc_batch_*):
 *   out_j[0 .. len_j) = sum_{t in job j} coef_t * src_t[0 .. len_t)   (src zero-extended past len_t)
 * and, when out2_j != 0, the same bytes at out2_j too.  jobs [njobs] and terms (indexed by the
 * jobs) are device arrays; src / out / out2 are device addresses or pinned host memory
 * (hipHostMalloc: the adaptor reads this flush's new payloads and writes the results it hands to
 * callbacks there, with no copy engine in between), 16-byte aligned with readable / writable
 * bytes up to len rounded up to 16 (outputs are zero-padded there); len_t <= len_j;
 * max_len >= every len_j.  One wave per (job, 1 KiB of output).
 * Replaces, for a whole batch flush, the per-operation region calls of detail/encoder.cc:15-64
 * and detail/decoder.cc:156-178, 393-408, 503-534. */
typedef struct {
  uint64_t out;          /* address of the output payload */
  uint64_t out2;         /* 0, or a second address receiving the same bytes */
  uint32_t term0;        /* first term of this job */
  uint32_t nterms;
  uint32_t len;          /* output bytes (<= 65535) */
  uint32_t pad;
} ntc_gf256_gather_job;
typedef struct {
  uint64_t src;          /* address of an input payload */
  uint32_t len;          /* bytes of it that take part */
  uint32_t coef;         /* GF(2^8) coefficient (low byte) */
} ntc_gf256_gather_term;
int  ntc_gf256_gather_combine(ntc_gf256_engine* eng, uint32_t njobs, const ntc_gf256_gather_job* jobs,
                              const ntc_gf256_gather_term* terms, uint32_t max_len, void* stream);

/* ---- Dense codes: caller-supplied coefficient matrices (BASELINE config 5 extension) --------
 * The reference's w = 8 schedule cannot build large invertible systems (coefficient() has period
 * 255), so k = 1024 "all sources lost" decoding uses a dense matrix chosen by the caller.
 * mat [G][n][n] row-major, row j = coefficients of repair j over sources 0..n-1 (rep = mat * src).
 *
 * ntc_gf256_dense_invert_batch  <- ntc::detail::invert (invert_matrix.cc:9-128) for n <= 1024:
 *   inv [G][n][n] = mat^-1 (the inverse is unique; device blocked Gauss-Jordan).  ok[g] = 1 if
 *   mat[g] is invertible, 0 if singular (inv[g] is then all zero).  ok may be NULL.
 * ntc_gf256_dense_encode_batch  <- detail::encoder (encoder.cc:15-64) with mat [G][r][k] in place
 *   of the coefficient schedule: rep[g][j] = sum_i mat[g][j][i] * src[g][i] over `stride` bytes.
 * ntc_gf256_dense_decode_batch  <- attempt_full_decoding's invert + MAC (decoder.cc:412-534):
 *   out[g] = mat[g]^-1 * rep[g] ([G][n][stride]); ok[g] as above (out[g] zero when singular). */
int  ntc_gf256_dense_invert_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t n,
                                  const uint8_t* mat, uint8_t* inv, uint8_t* ok, void* stream);
int  ntc_gf256_dense_encode_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                                  uint32_t stride, const uint8_t* mat, const uint8_t* src,
                                  uint8_t* rep, void* stream);
int  ntc_gf256_dense_decode_batch(ntc_gf256_engine* eng, uint32_t G, uint32_t n, uint32_t stride,
                                  const uint8_t* mat, const uint8_t* rep, uint8_t* out,
                                  uint8_t* ok, void* stream);

/* ---- Wire format on the device (netcode/detail/packetizer.hh) ---------------------------------
 * Packets live in fixed-size slots: packet p at pkts + p * pkt_stride (a multiple of 16), its
 * length in pkt_len[p] -- the shape of a sendmmsg / recvmmsg batch.  Integers big-endian.
 *
 * ntc_gf256_write_repairs  <- packetizer::write_repair (packetizer.hh:90-122), called by
 *   ntc::encoder::generate_repair (encoder.hh:321-333) once per repair: packet (g, j) =
 *   [u8 1][u32 rid_base[g]+j][u16 rep_len[g]][symbol][ids][u16 rep_size[g][j]][u16 rep_len[g]]
 *   [symbol] with ids = the generation's k source ids in write_ids' run-length form (:263-309).
 *   rep/rep_size/rep_len as produced by ntc_gf256_encode_batch.  pkt_stride >=
 *   ntc_gf256_repair_packet_bytes(k, stride).
 * ntc_gf256_write_sources  <- packetizer::write_source (:165-183), called by ntc::encoder::
 *   operator()(data) for systematic codes (encoder.hh:255-285): packet (g, i) =
 *   [u8 2][u32 sid_base[g]+i][u16 src_len[g][i]][payload].  pkt_stride >= 7 + stride.
 * ntc_gf256_read_packets   <- ntc::decoder::operator()(packet) (decoder.hh: get_packet_type
 *   dispatch) + packetizer::read_source / read_repair (:125-158, 186-218): each packet is parsed
 *   and its symbol scattered into the batch layout of ntc_gf256_decode_batch -- source id s to
 *   slot (s - sid0) of src [G*k], repair id q to slot (q - rid0) of rep [G*r] (generation
 *   g = slot / k or slot / r, i.e. sid_base[g] = sid0 + g*k, rid_base[g] = rid0 + g*r), zero-padded
 *   to stride; src_len / src_mask / rep_size / rep_mask filled.  The call first zeroes the four
 *   per-slot arrays (slots of packets not received keep their old bytes).  status[p] is one of
 *   NTC_PKT_*; only NTC_PKT_SOURCE / NTC_PKT_REPAIR packets are stored.  A repair is stored only
 *   when its id list is exactly its generation's k consecutive source ids (the batched decoder's
 *   model).  Duplicate packets must carry identical bytes. */
enum {
  NTC_PKT_SOURCE = 0,          /* stored into src */
  NTC_PKT_REPAIR = 1,          /* stored into rep */
  NTC_PKT_ACK = 2,             /* an ack (type 0): not data, skipped */
  NTC_PKT_BAD_TYPE = 3,        /* unknown type byte (reference: packet_type_error) */
  NTC_PKT_OVERFLOW = 4,        /* truncated packet (reference: overflow_error) */
  NTC_PKT_OUT_OF_BATCH = 5,    /* id outside [sid0, sid0 + G*k) / [rid0, rid0 + G*r) */
  NTC_PKT_TOO_LARGE = 6,       /* symbol longer than stride */
  NTC_PKT_NOT_GENERATION = 7   /* repair not over exactly its generation's k sources */
};
uint32_t ntc_gf256_repair_packet_bytes(uint32_t k, uint32_t stride);
int  ntc_gf256_write_repairs(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t r,
                             uint32_t stride, const uint8_t* rep, const uint16_t* rep_size,
                             const uint16_t* rep_len, const uint32_t* sid_base,
                             const uint32_t* rid_base, uint8_t* out, uint32_t pkt_stride,
                             uint32_t* pkt_len, void* stream);
int  ntc_gf256_write_sources(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t stride,
                             const uint8_t* src, const uint16_t* src_len, const uint32_t* sid_base,
                             uint8_t* out, uint32_t pkt_stride, uint32_t* pkt_len, void* stream);
int  ntc_gf256_read_packets(ntc_gf256_engine* eng, uint32_t npkts, const uint8_t* pkts,
                            uint32_t pkt_stride, const uint32_t* pkt_len, uint32_t G, uint32_t k,
                            uint32_t r, uint32_t stride, uint32_t sid0, uint32_t rid0,
                            uint8_t* src, uint16_t* src_len, uint8_t* src_mask, uint8_t* rep,
                            uint16_t* rep_size, uint8_t* rep_mask, uint8_t* status, void* stream);
/* The same without the reset: the packets of a further recvmmsg batch (e.g. another packet size's
 * slots) are added to what earlier read_packets / read_packets_append calls stored. */
int  ntc_gf256_read_packets_append(ntc_gf256_engine* eng, uint32_t npkts, const uint8_t* pkts,
                                   uint32_t pkt_stride, const uint32_t* pkt_len, uint32_t G,
                                   uint32_t k, uint32_t r, uint32_t stride, uint32_t sid0,
                                   uint32_t rid0, uint8_t* src, uint16_t* src_len, uint8_t* src_mask,
                                   uint8_t* rep, uint16_t* rep_size, uint8_t* rep_mask,
                                   uint8_t* status, void* stream);

/* ---- Packed rows <-> generation slots (host-resident batches) ---------------------------------
 * A receiver holds only the sources it received and wants back only the ones it lost; these two
 * byte movers let a host-resident caller ship exactly those over PCIe (the reference's decoder
 * likewise stores received sources and hands out only recovered ones, decoder.hh: data_handler).
 * Slot (g, i) is *selected* when (mask[g][i] != 0) == want; the selected slots of generation g
 * map, in slot order, to packed rows row_base[g] - row0, row_base[g] - row0 + 1, ... of `packed`
 * ([rows][stride]; row_base = the caller's prefix sum of selected counts, row0 lets a chunk of a
 * batch use the batch's row_base with a chunk-relative packed buffer).
 * ntc_gf256_unpack_slots  packed rows -> selected slots of slots [G][k][stride]; zero_rest != 0
 *                         zeroes every slot that is not selected (e.g. the lost ones, so a
 *                         generation that does not decode returns zeros).
 * ntc_gf256_pack_slots    selected slots -> packed rows (e.g. want = 0: the recovered sources
 *                         after ntc_gf256_decode_batch). */
int  ntc_gf256_unpack_slots(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t stride,
                            const uint8_t* packed, const uint32_t* row_base, uint32_t row0,
                            const uint8_t* mask, uint8_t want, uint8_t* slots, int zero_rest,
                            void* stream);
int  ntc_gf256_pack_slots(ntc_gf256_engine* eng, uint32_t G, uint32_t k, uint32_t stride,
                          const uint8_t* slots, const uint8_t* mask, uint8_t want,
                          const uint32_t* row_base, uint32_t row0, uint8_t* packed, void* stream);

/* dst = c*src (add = 0) or dst ^= c*src (add = 1) over `len` bytes of device memory. */
int  ntc_gf256_region_multiply(ntc_gf256_engine* eng, const uint8_t* src, uint8_t* dst,
                               size_t len, uint8_t c, int add, void* stream);

/* ---- GF(2^w) for every field size netcode supports, w in {4, 8, 16, 32} --------------------
 * galois_field.hh:35-44 gf_init_easy(&gf, w) -- gf-complete's default fields: primitive
 * polynomials 0x13 (w=4), 0x11D (w=8), 0x1100B (w=16), x^32 + 0x400007 (w=32).  Regions follow
 * multiply_region.w32: w=4 multiplies every nibble, w=8 every byte, w=16 / w=32 every
 * little-endian 16- / 32-bit word (a partial last word reads missing bytes as zero and writes
 * only bytes inside the region).  Coefficients are field elements (< 2^w).
 *
 * ntc_gf_combine_batch   <- the region MACs of detail/encoder.cc:15-64 and detail/decoder.cc
 *   (:156-178, 393-408, 480-559) for any w: out[g][j] = sum_i coef[g][i][j] * in[g][i] over
 *   `stride` bytes (stride a multiple of 16), coef [G][k][rows] u32.
 * ntc_gf_region_multiply <- galois_field::multiply / multiply_add (galois_field.hh:65-92).
 * ntc_gf_coefficient / ntc_gf_multiply / ntc_gf_invert / ntc_gf_multiply_size  <-
 *   galois_field::coefficient (:143-158, w = 32: the raw uint32 product, 0 -> 1), multiply
 *   (:123-130), invert (:133-139), multiply_size (:96-120; w = 32 truncates to 16 bits, :118).
 *   Host-side, no device work; they return 0 for an unsupported w. */
int  ntc_gf_combine_batch(ntc_gf256_engine* eng, uint32_t w, uint32_t G, uint32_t k, uint32_t rows,
                          uint32_t stride, const uint8_t* in, const uint32_t* coef, uint8_t* out,
                          void* stream);
int  ntc_gf_region_multiply(ntc_gf256_engine* eng, uint32_t w, const uint8_t* src, uint8_t* dst,
                            size_t len, uint32_t c, int add, void* stream);
uint32_t ntc_gf_coefficient(uint32_t w, uint32_t repair_id, uint32_t src_id);
uint32_t ntc_gf_multiply(uint32_t w, uint32_t x, uint32_t y);
uint32_t ntc_gf_invert(uint32_t w, uint32_t x);
uint16_t ntc_gf_multiply_size(uint32_t w, uint16_t size, uint32_t coeff);

/* Host-side scalar helpers (no device work). */
uint32_t ntc_gf256_coefficient(uint32_t repair_id, uint32_t src_id);
uint16_t ntc_gf256_multiply_size(uint16_t size, uint32_t coeff);
uint8_t  ntc_gf256_multiply(uint8_t x, uint8_t y);
uint8_t  ntc_gf256_invert(uint8_t x);

/* Thread-local description of the last error on this thread ("" if none). */
const char* ntc_gf256_last_error(void);

/* Build description: "gfx950 ..." (lets callers check the native library really loaded). */
const char* ntc_gf256_build_info(void);

#ifdef __cplusplus
}
#endif
#endif
