/* Per-packet workload through the reference's C ABI (libntc.so: the include/netcode/c headers,
 * batching from netcode/c/ext.h), the GPU side of bench.py --per-packet at C level.
 *
 * F flows x M items of S bytes, one encoder per flow (window W, a repair every R sources), fed
 * round-robin (one ntc_encoder_add_data per item and flow); then each flow's packets minus an
 * i.i.d. L % loss into its own in-order decoder, round-robin, one ntc_decoder_add_packet each.
 * Payloads and losses are drawn exactly as the CPU leg draws them (or_pp_bench in the oracle), so
 * both must produce the same packets and deliveries (FNV-1a hashes).  mode "batched": every
 * encoder / decoder attached to one ntc_batch_t, flushed once per round (decoders every 4 rounds
 * and at the end).  Prints one JSON object.
 *
 * usage: pp_driver <immediate|batched|async> F M S W R L seed
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "netcode/c/data.h"
#include "netcode/c/decoder.h"
#include "netcode/c/encoder.h"
#include "netcode/c/ext.h"
#include "netcode/c/packet.h"

static uint64_t mix(uint64_t x)
{
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

static uint64_t fnv(uint64_t h, const uint8_t* p, size_t n)
{
  for (size_t i = 0; i < n; ++i) h = (h ^ p[i]) * 0x100000001B3ull;
  return h;
}

typedef struct {
  uint8_t* v;
  size_t n, cap;
  size_t* off;
  size_t np, capp;
} store;

static void append(store* s, const char* p, size_t n)
{
  if (s->n + n > s->cap) {
    s->cap = (s->n + n) * 2 + 4096;
    s->v = (uint8_t*)realloc(s->v, s->cap);
  }
  memcpy(s->v + s->n, p, n);
  s->n += n;
}

static void close_item(store* s)
{
  if (s->np + 2 > s->capp) {
    s->capp = s->capp * 2 + 64;
    s->off = (size_t*)realloc(s->off, s->capp * sizeof(size_t));
  }
  if (s->np == 0) s->off[0] = 0;
  s->off[++s->np] = s->n;
}

static void on_prepare(void* ctx, const char* p, size_t n) { append((store*)ctx, p, n); }
static void on_send(void* ctx) { close_item((store*)ctx); }
static void on_data(void* ctx, const char* p, size_t n)
{
  append((store*)ctx, p, n);
  close_item((store*)ctx);
}

static double now(void)
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* tools/sampler.c, when preloaded with NTC_SAMPLER_GATED=1, records only inside the timed loops;
 * PP_PROFILE=enc or dec narrows that to one of them */
static void prof_gate(int on, const char* phase)
{
  static void (*f)(int) = NULL;
  static int looked = 0;
  if (!looked) {
    f = (void (*)(int))dlsym(RTLD_DEFAULT, "ntc_sampler_enable");
    looked = 1;
  }
  const char* want = getenv("PP_PROFILE");
  if (f && (!want || strcmp(want, phase) == 0)) f(on);
}

static int check(const ntc_error* e, const char* what)
{
  if (e->type != ntc_no_error) {
    fprintf(stderr, "pp_driver: %s failed (type %d)\n", what, (int)e->type);
    return 1;
  }
  return 0;
}

int main(int argc, char** argv)
{
  if (argc != 9) {
    fprintf(stderr, "usage: %s <immediate|batched|async> F M S W R L seed\n", argv[0]);
    return 2;
  }
  /* "async": batched, with asynchronous flushes (each flush's GPU work overlaps the next round) */
  const int async = strcmp(argv[1], "async") == 0;
  const int batched = async || strcmp(argv[1], "batched") == 0;
  const uint32_t F = (uint32_t)atoi(argv[2]), M = (uint32_t)atoi(argv[3]), S = (uint32_t)atoi(argv[4]);
  const uint32_t W = (uint32_t)atoi(argv[5]), R = (uint32_t)atoi(argv[6]), L = (uint32_t)atoi(argv[7]);
  const uint64_t seed = strtoull(argv[8], NULL, 10);
  ntc_error err;
  uint8_t* data = (uint8_t*)malloc((size_t)M * S + 8);
  for (uint32_t i = 0; i < M; ++i)
    for (uint32_t b = 0; b < S; ++b)
      data[(size_t)i * S + b] = (uint8_t)(mix(seed + ((uint64_t)i << 32) + b / 8) >> (8 * (b % 8)));
  store* tx = (store*)calloc(F, sizeof(store));
  store* rx = (store*)calloc(F, sizeof(store));
  store* acks = (store*)calloc(F, sizeof(store));
  ntc_encoder_t** enc = (ntc_encoder_t**)calloc(F, sizeof(void*));
  ntc_decoder_t** dec = (ntc_decoder_t**)calloc(F, sizeof(void*));
  ntc_batch_t* eb = batched ? ntc_new_batch() : NULL;
  ntc_batch_t* db = batched ? ntc_new_batch() : NULL;
  ntc_batch_set_eager(eb, 1);        /* source packets and received deliveries go out at once */
  ntc_batch_set_eager(db, 1);
  ntc_batch_set_async(eb, async);
  ntc_batch_set_async(db, async);
  for (uint32_t f = 0; f < F; ++f) {
    ntc_packet_handler h = {&tx[f], on_prepare, on_send};
    enc[f] = ntc_new_encoder(8, h);
    if (!enc[f]) {
      fprintf(stderr, "pp_driver: no encoder (no MI355X engine?)\n");
      return 1;
    }
    ntc_encoder_set_rate(enc[f], R);
    ntc_encoder_set_window_size(enc[f], W);
    if (eb) {
      ntc_encoder_set_batch(enc[f], eb, &err);
      if (check(&err, "ntc_encoder_set_batch")) return 1;
    }
  }
  for (uint32_t f = 0; f < F; ++f) {     /* stores sized and paged in before the clock (as or_pp_bench) */
    tx[f].cap = (size_t)M * (S + 16) + (size_t)((R ? M / R : M) + 1) * (2 * S + 256);
    tx[f].v = (uint8_t*)calloc(tx[f].cap, 1);
    memset(tx[f].v, 0, tx[f].cap);
    tx[f].capp = 2 * (size_t)M + 64;
    tx[f].off = (size_t*)malloc(tx[f].capp * sizeof(size_t));
    rx[f].cap = (size_t)M * S + 4096;
    rx[f].v = (uint8_t*)calloc(rx[f].cap, 1);
    memset(rx[f].v, 0, rx[f].cap);
    rx[f].capp = (size_t)M + 64;
    rx[f].off = (size_t*)malloc(rx[f].capp * sizeof(size_t));
  }
  /* one data object per flow, filled inside the loop like an application producing its items (the
   * encoder takes the buffer; the object is refilled for the next item) -- the CPU leg copies each
   * item into its window the same way */
  ntc_data_t** items = (ntc_data_t**)calloc(F, sizeof(void*));
  for (uint32_t f = 0; f < F; ++f) items[f] = ntc_new_data(0);
  double t_flush_enc = 0, t_flush_dec = 0;   /* time inside ntc_batch_flush (GPU round trips) */
  prof_gate(1, "enc");
  double t0 = now();
  for (uint32_t i = 0; i < M; ++i) {
    for (uint32_t f = 0; f < F; ++f) {
      ntc_data_resize(items[f], (uint16_t)S, &err);
      if (check(&err, "ntc_data_resize")) return 1;
      memcpy(ntc_data_buffer(items[f]), data + (size_t)i * S, S);
      ntc_encoder_add_data(enc[f], items[f], &err);
      if (check(&err, "ntc_encoder_add_data")) return 1;
    }
    if (eb) {
      const double tf = now();
      ntc_batch_flush(eb, &err);
      t_flush_enc += now() - tf;
      if (check(&err, "ntc_batch_flush")) return 1;
    }
  }
  if (eb)                           /* async: the last flush's events (a no-op otherwise) */
    while (ntc_batch_pending(eb)) {
      const double tf = now();
      ntc_batch_flush(eb, &err);
      t_flush_enc += now() - tf;
      if (check(&err, "ntc_batch_flush")) return 1;
    }
  const double t_enc = now() - t0;
  prof_gate(0, "enc");
  uint64_t npk = 0, nrep = 0, nrx = 0, ndel = 0;
  for (uint32_t f = 0; f < F; ++f) {
    npk += tx[f].np;
    nrep += ntc_encoder_counter(enc[f], NTC_ENC_NB_SENT_REPAIRS);
  }
  /* received streams (or_pp_bench's loss draw), as packet objects made before the clock starts */
  uint32_t* nkeep = (uint32_t*)calloc(F, sizeof(uint32_t));
  ntc_packet_t*** pk = (ntc_packet_t***)calloc(F, sizeof(void*));
  uint32_t rounds = 0;
  for (uint32_t f = 0; f < F; ++f) {
    pk[f] = (ntc_packet_t**)calloc(tx[f].np + 1, sizeof(void*));
    for (uint32_t j = 0; j < tx[f].np; ++j)
      if (mix(seed ^ 0x5EEDull ^ ((uint64_t)f << 40) ^ j) % 100 >= L)
        pk[f][nkeep[f]++] = ntc_new_packet_from((const char*)tx[f].v + tx[f].off[j],
                                                (uint16_t)(tx[f].off[j + 1] - tx[f].off[j]));
    nrx += nkeep[f];
    if (nkeep[f] > rounds) rounds = nkeep[f];
    ntc_packet_handler ph = {&acks[f], on_prepare, on_send};
    ntc_data_handler dh = {&rx[f], on_data};
    dec[f] = ntc_new_decoder(8, ntc_in_order_yes, ph, dh);
    if (!dec[f]) return 1;
    ntc_decoder_set_ack_period(dec[f], 0);
    if (db) {
      ntc_decoder_set_batch(dec[f], db, &err);
      if (check(&err, "ntc_decoder_set_batch")) return 1;
    }
  }
  prof_gate(1, "dec");
  t0 = now();
  for (uint32_t i = 0; i < rounds; ++i) {
    for (uint32_t f = 0; f < F; ++f)
      if (i < nkeep[f]) {
        ntc_decoder_add_packet(dec[f], pk[f][i], &err);
        if (check(&err, "ntc_decoder_add_packet")) return 1;
      }
    if (db && i % 4 == 3) {
      const double tf = now();
      ntc_batch_flush(db, &err);
      t_flush_dec += now() - tf;
      if (check(&err, "ntc_batch_flush")) return 1;
    }
  }
  if (db)
    do {                            /* async: until the last flush's events are delivered */
      const double tf = now();
      ntc_batch_flush(db, &err);
      t_flush_dec += now() - tf;
      if (check(&err, "ntc_batch_flush")) return 1;
    } while (ntc_batch_pending(db));
  const double t_dec = now() - t0;
  prof_gate(0, "dec");
  uint64_t hp = 0xCBF29CE484222325ull, hd = 0xCBF29CE484222325ull;
  for (uint32_t f = 0; f < F; ++f) {
    hp = fnv(hp, tx[f].v, tx[f].n);
    hd = fnv(hd, rx[f].v, rx[f].n);
    ndel += rx[f].np;
  }
  printf("{\"mode\": \"%s\", \"encode_s\": %.6f, \"decode_s\": %.6f, \"encode_flush_s\": %.6f, "
         "\"decode_flush_s\": %.6f, \"packets\": %llu, "
         "\"received\": %llu, \"deliveries\": %llu, \"repairs\": %llu, "
         "\"packets_hash\": \"%016llx\", \"deliveries_hash\": \"%016llx\"}\n",
         argv[1], t_enc, t_dec, t_flush_enc, t_flush_dec, (unsigned long long)npk, (unsigned long long)nrx,
         (unsigned long long)ndel, (unsigned long long)nrep, (unsigned long long)hp,
         (unsigned long long)hd);
  for (uint32_t f = 0; f < F; ++f) {
    for (uint32_t i = 0; i < nkeep[f]; ++i) ntc_delete_packet(pk[f][i]);
    free(pk[f]);
    ntc_delete_encoder(enc[f]);
    ntc_delete_decoder(dec[f]);
    free(tx[f].v); free(tx[f].off); free(rx[f].v); free(rx[f].off); free(acks[f].v); free(acks[f].off);
  }
  for (uint32_t f = 0; f < F; ++f) ntc_delete_data(items[f]);
  ntc_delete_batch(eb);
  ntc_delete_batch(db);
  free(items); free(pk); free(nkeep); free(tx); free(rx); free(acks); free(enc); free(dec); free(data);
  return 0;
}
