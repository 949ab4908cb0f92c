/*
 * ntc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of ahamez/netcode's GF(2^8) coding path (reference at /root/reference, read
 * only).  This is the *checker*: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load it.  The product (netcode_amd/, libntc_gf256.so) never links or calls it.
 *
 * Parity pins (see DESIGN.md "Oracle"):
 *   - GF(2^8) polynomial 0x11D (gf-complete's w=8 default; the reference calls gf_init_easy(&gf,8)
 *     at netcode/detail/galois_field.hh:40 and never names the polynomial).
 *   - SURVEY.md §8(c) hand-checked KATs (wire bytes of a 2-source repair, scalar coefficients,
 *     inverses) and SURVEY.md §6 end_to_end golden counters (reference compiled in the survey
 *     container, 1000 and 10000 packets).
 *   - tests/netcode/detail/test_invert_matrix.cc (jerasure inverse equality, singular 3x3).
 */
#ifndef NTC_ORACLE_H
#define NTC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- GF(2^8) / 0x11D ---------- */
uint8_t  or_gf_mul(uint8_t a, uint8_t b);
/* These run in the calling thread's field (GF(2^8) unless or_set_field chose another). */
uint32_t or_gf_inv(uint32_t a);                   /* a != 0 */
uint32_t or_coefficient(uint32_t repair_id, uint32_t src_id);   /* galois_field.hh:143-158 */
void     or_region_mul(const uint8_t* src, uint8_t* dst, size_t len, uint32_t c);
void     or_region_muladd(const uint8_t* src, uint8_t* dst, size_t len, uint32_t c);
uint16_t or_multiply_size(uint16_t size, uint32_t c);           /* galois_field.hh:96-120 */

/* Jerasure Gauss-Jordan on a column-major square_matrix (invert_matrix.cc:9-128).
 * Returns -1 on success, else the failure index the reference returns (rows-1). */
long     or_invert(uint32_t* mat, uint32_t* inv, size_t n);

/* ------------------------------------------------ dense codes (BASELINE config 5 extension) ---- */
/* No reference counterpart beyond its building blocks: mat is a caller-chosen dense matrix (the
 * reference's w=8 schedule makes k > 255 systems singular).  rep[j] = sum_i mat[j][i] * src[i]
 * (mat [r][k] row-major, region MACs of galois_field.hh:83-92). */
void or_dense_encode(uint32_t k, uint32_t r, size_t stride, const uint8_t* mat, const uint8_t* src,
                     uint8_t* rep);
/* out = mat^-1 * rep via or_invert (invert_matrix.cc:9-128) + region MACs (decoder.cc:503-534).
 * Returns -1 on success, else or_invert's failure index (out and inv zeroed).  inv [n][n] row-major
 * may be NULL. */
long or_dense_decode(uint32_t n, size_t stride, const uint8_t* mat, const uint8_t* rep, uint8_t* out,
                     uint8_t* inv);

/* -------------------------------------------------------- generation encode (batch form) ---- */
/* One generation: R_j = sum_i c(rid_base+j, sid_base+i) * X_i, sources zero padded to `stride`
 * (detail/encoder.cc:15-64).  src: [k][stride], rep: [r][stride]; rep_size[j] = encoded size. */
void or_encode_generation(uint32_t k, uint32_t r, uint32_t stride, const uint8_t* src,
                          const uint16_t* src_len, uint32_t sid_base, uint32_t rid_base,
                          uint8_t* rep, uint16_t* rep_size, uint16_t* rep_len);

/* Batch encode over G generations, optional OpenMP-free pthread fan-out (nthreads >= 1). */
void or_encode_batch(uint32_t G, uint32_t k, uint32_t r, uint32_t stride, const uint8_t* src,
                     const uint16_t* src_len, const uint32_t* sid_base, const uint32_t* rid_base,
                     uint8_t* rep, uint16_t* rep_size, int use_simd, int nthreads);

/* -------------------------------------------------------- generation decode (batch form) ---- */
/* Per-generation result of feeding the received sources (ascending id) then the received
 * repairs (ascending id) of one generation into a fresh reference decoder
 * (detail/decoder.cc:33-152, 412-566). */
typedef struct {
  uint8_t  state;          /* 0 decoded, 1 nothing missing, 2 not enough repairs, 3 singular */
  uint8_t  nb_failed;      /* nb_failed_full_decodings */
  uint16_t nb_missing;     /* m */
  uint16_t nb_decoded;     /* nb_decoded */
  uint16_t nb_useless;     /* nb_useless_repairs */
  uint16_t last_repair;    /* index (in the generation) of the repair that completed decoding */
  uint16_t pad;
} or_decode_status;

/* src: [k][stride] in/out (lost slots receive recovered payloads zero-padded to stride);
 * src_len in/out; rep: [r][stride]; rep_size: encoded sizes; masks: 1 = received. */
void or_decode_generation(uint32_t k, uint32_t r, uint32_t stride, uint8_t* src, uint16_t* src_len,
                          const uint8_t* src_mask, const uint8_t* rep, const uint16_t* rep_size,
                          const uint16_t* rep_len, const uint8_t* rep_mask, uint32_t sid_base,
                          uint32_t rid_base, or_decode_status* st);

void or_decode_batch(uint32_t G, uint32_t k, uint32_t r, uint32_t stride, uint8_t* src,
                     uint16_t* src_len, const uint8_t* src_mask, const uint8_t* rep,
                     const uint16_t* rep_size, const uint16_t* rep_len, const uint8_t* rep_mask,
                     const uint32_t* sid_base, const uint32_t* rid_base, or_decode_status* st,
                     int use_simd, int nthreads);

/* ----------------------------------------------------- streaming protocol (packet level) ---- */
typedef struct or_encoder or_encoder;
typedef struct or_decoder or_decoder;

/* Packets are delivered to `emit(ctx, bytes, len)` as whole wire packets. */
typedef void (*or_emit_fn)(void* ctx, const uint8_t* bytes, size_t len);
/* Decoded / received sources are delivered to `deliver(ctx, id, bytes, len)`. */
typedef void (*or_deliver_fn)(void* ctx, uint32_t id, const uint8_t* bytes, size_t len);

or_encoder* or_encoder_new(or_emit_fn emit, void* ctx);
void        or_encoder_free(or_encoder*);
void        or_encoder_set_field(or_encoder*, int w);   /* galois_field_size, default 8 */
void        or_encoder_set_rate(or_encoder*, size_t rate);
void        or_encoder_set_window_size(or_encoder*, size_t sz);
void        or_encoder_set_code_type(or_encoder*, int systematic);
void        or_encoder_set_adaptive(or_encoder*, int adaptive);
void        or_encoder_add_data(or_encoder*, const uint8_t* data, uint16_t len);
long        or_encoder_add_packet(or_encoder*, const uint8_t* pkt, size_t len); /* -1: type err */
void        or_encoder_generate_repair(or_encoder*);
size_t      or_encoder_window(const or_encoder*);
size_t      or_encoder_rate(const or_encoder*);
size_t      or_encoder_nb_sent_repairs(const or_encoder*);
size_t      or_encoder_nb_sent_sources(const or_encoder*);
size_t      or_encoder_nb_received_acks(const or_encoder*);

or_decoder* or_decoder_new(int in_order, or_emit_fn emit, void* ectx, or_deliver_fn deliver,
                           void* dctx);
void        or_decoder_set_field(or_decoder*, int w);
void        or_decoder_free(or_decoder*);
long        or_decoder_add_packet(or_decoder*, const uint8_t* pkt, size_t len); /* -1: err */
void        or_decoder_generate_ack(or_decoder*);
void        or_decoder_set_ack_nb_packets(or_decoder*, uint16_t nb);
void        or_decoder_set_ack_period_ms(or_decoder*, long ms);  /* 0 disables timed acks */
size_t      or_decoder_counter(const or_decoder*, int which);
/* which: 0 nb_decoded, 1 nb_failed_full_decodings, 2 nb_missing_sources, 3 nb_received_repairs,
 *        4 nb_received_sources, 5 nb_sent_acks, 6 nb_useless_repairs, 7 nb_repairs_pending */

/* tests/end_to_end.cc:90-201 restated: 1024-B payloads, GF(256), rate 5, in-order decoder, ack
 * every 50 received packets, loss::burst{95,5} (tools/loss/burst.hh) shared by both directions.
 * out[0..6] = sent, lost(to decoder), received repairs, received sources, useless, decoded,
 * handled data.  Returns 0 on success, -1 if the in-order data check fails. */
int or_end_to_end(uint32_t nb_packets, uint64_t* out);

/* loss models: libstdc++ std::default_random_engine (minstd_rand0, seed 1) +
 * uniform_int_distribution<unsigned>{1,100} (tools/loss/{burst,uniform}.hh). */
typedef struct { uint32_t state; int bad; unsigned good_th, bad_th; } or_burst;
void or_burst_init(or_burst*, unsigned good, unsigned bad);
int  or_burst_next(or_burst*);           /* 1 = lost */
typedef struct { uint32_t state; unsigned threshold; } or_uniform;
void or_uniform_init(or_uniform*, unsigned threshold);
int  or_uniform_next(or_uniform*);       /* 1 = lost */

/* AVX2 split-nibble region MAC: the algorithm class of gf-complete's w=8 default (SPLIT 8,4
 * with pshufb); used as the CPU baseline.  Falls back to the scalar loop without AVX2. */
void or_region_muladd_simd(const uint8_t* src, uint8_t* dst, size_t len, uint8_t c);
int  or_have_avx2(void);
int  or_have_gfni(void);               /* GFNI + AVX-512BW region path available (or_set_simd(2)) */
/* Route the oracle's own region ops through the AVX2 kernel (CPU baseline timing only). */
void or_set_simd(int on);

/* GF(2^w), w in {4, 8, 16, 32}: gf-complete's default polynomials 0x13 / 0x11D / 0x1100B /
 * 0x400007 (galois_field.hh:35-44 gf_init_easy); region semantics per nibble / byte / LE u16 /
 * LE u32 word; multiply_size per galois_field.hh:96-120 (w = 32 truncated). */
void     or_set_field(int w);                      /* this thread's field for the calls above */
int      or_field(void);
uint32_t or_fw_mul(int w, uint32_t a, uint32_t b);
uint32_t or_fw_inv(int w, uint32_t a);
uint32_t or_fw_coefficient(int w, uint32_t repair_id, uint32_t src_id);
void     or_fw_region(int w, const uint8_t* src, uint8_t* dst, size_t len, uint32_t c, int add);
uint16_t or_fw_multiply_size(int w, uint16_t size, uint32_t c);

/* Wire format (packetizer.hh:90-122, 165-183) and one packet's ingestion into a batch layout
 * (the specification of ntc_gf256_read_packets; status codes NTC_PKT_* of netcode/gpu.h). */
size_t or_write_repair_packet(uint32_t rid, const uint8_t* sym, uint16_t symsz, const uint32_t* ids,
                              size_t n, uint16_t esz, uint8_t* out);
size_t or_write_source_packet(uint32_t sid, const uint8_t* data, uint16_t len, uint8_t* out);
int or_read_packet_into(const uint8_t* pkt, size_t len, uint32_t G, uint32_t k, uint32_t r,
                        uint32_t stride, uint32_t sid0, uint32_t rid0, uint8_t* src,
                        uint16_t* src_len, uint8_t* src_mask, uint8_t* rep, uint16_t* rep_size,
                        uint8_t* rep_mask);

/* --------------------------------------- packet-level pieces for tests/oracle_surface ------ */
/* The reference's detail layer over this restatement (tests only): the reference's own Catch suites
 * and end_to_end.cc compile against the headers under tests/oracle_surface/ and run HERE, so the checker is
 * pinned by the reference's own expectations. */
typedef struct {
  uint8_t  type;            /* 0 ack, 1 repair, 2 source */
  uint32_t id;              /* repair / source id */
  uint16_t nb_packets;      /* ack */
  uint16_t encoded_size;    /* repair */
  uint16_t symbol_size;     /* repair / source */
  size_t   symbol_offset;   /* the (first) symbol copy, from the packet start */
  uint32_t* ids; size_t nids;   /* ack / repair: sorted unique source ids (malloc'd) */
} or_packet_view;
long   or_parse_packet(const uint8_t* pkt, size_t len, or_packet_view* out);  /* -1 type, -2 overflow */
void   or_packet_view_free(or_packet_view*);
size_t or_write_ack_packet(uint16_t nb_packets, const uint32_t* ids, size_t n, uint8_t* out);
size_t or_packet_bound(size_t symsz, size_t nids);     /* bytes a repair / ack packet may need */
/* detail/encoder.cc:15-64 in field w: returns the repair symbol length (max of lens). */
uint16_t or_build_repair(int w, uint32_t rid, size_t n, const uint32_t* ids, const uint8_t* const* syms,
                         const uint16_t* lens, uint8_t* sym, uint16_t* esz);
void   or_decoder_maybe_ack(or_decoder*);           /* decoder.hh:231-248 */

/* detail::decoder (detail/decoder.hh) as an object: the streaming core the public decoder and
 * or_decode_batch run. */
typedef struct or_dcore or_dcore;
typedef void (*or_source_fn)(void* ctx, uint32_t id, const uint8_t* bytes, uint16_t len);
or_dcore* or_dcore_new(int w, int in_order, or_source_fn cb, void* ctx);
void      or_dcore_free(or_dcore*);
void      or_dcore_add_source(or_dcore*, uint32_t id, const uint8_t* data, uint16_t len);
void      or_dcore_add_repair(or_dcore*, uint32_t id, const uint32_t* ids, size_t n, uint16_t esz,
                              const uint8_t* sym, uint16_t symsz);
uint16_t  or_dcore_create_source_from_repair(or_dcore*, uint32_t rid, uint32_t sid, uint16_t esz,
                                             const uint8_t* sym, uint16_t symsz, uint8_t* out);
void      or_dcore_remove_source_from_repair(or_dcore*, uint32_t sid, const uint8_t* sdata,
                                             uint16_t slen, uint32_t rid, uint16_t* esz, uint8_t* sym);
/* which: 0 sources, 1 repairs, 2 missing sources, 3 nb_decoded, 4 nb_failed, 5 nb_useless */
size_t    or_dcore_count(const or_dcore*, int which);
uint32_t  or_dcore_source(const or_dcore*, size_t i, const uint8_t** data, uint16_t* len);
uint32_t  or_dcore_repair(const or_dcore*, size_t i, const uint32_t** ids, size_t* n, uint16_t* esz,
                          const uint8_t** sym, uint16_t* symsz);
uint32_t  or_dcore_missing(const or_dcore*, size_t i, const uint32_t** rids, size_t* n);

/* bench.py --per-packet CPU leg (C level): see ntc_oracle.c.  secs[2], counts[4], hashes[2]. */
int or_pp_bench(uint32_t flows, uint32_t items, uint32_t size, uint32_t window, uint32_t rate,
                uint32_t loss_pct, uint64_t seed, double* secs, uint64_t* counts, uint64_t* hashes);

#ifdef __cplusplus
}
#endif
#endif
