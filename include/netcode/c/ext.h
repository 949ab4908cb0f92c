/* netcode/c/ext.h -- introspection extensions of the MI355X build (not in the reference C ABI).
 * Exposes the counters the reference keeps on ntc::encoder / ntc::decoder (encoder.hh:114-143,
 * decoder.hh:157-210) so C callers and tests can read them. */
#ifndef NETCODE_C_EXT_H
#define NETCODE_C_EXT_H
#include "netcode/c/decoder.h"
#include "netcode/c/encoder.h"
#ifdef __cplusplus
extern "C" {
#endif

enum {
  NTC_ENC_NB_SENT_REPAIRS = 0, NTC_ENC_NB_SENT_SOURCES = 1, NTC_ENC_NB_RECEIVED_ACKS = 2,
  NTC_ENC_RATE = 3, NTC_ENC_WINDOW = 4
};
enum {
  NTC_DEC_NB_DECODED = 0, NTC_DEC_NB_FAILED_FULL_DECODINGS = 1, NTC_DEC_NB_MISSING_SOURCES = 2,
  NTC_DEC_NB_RECEIVED_REPAIRS = 3, NTC_DEC_NB_RECEIVED_SOURCES = 4, NTC_DEC_NB_SENT_ACKS = 5,
  NTC_DEC_NB_USELESS_REPAIRS = 6, NTC_DEC_NB_PENDING_REPAIRS = 7
};

size_t ntc_encoder_counter(const ntc_encoder_t* enc, int which) NTC_C_NOEXCEPT NTC_C_NONNULL;
size_t ntc_decoder_counter(const ntc_decoder_t* dec, int which) NTC_C_NOEXCEPT NTC_C_NONNULL;

/* Online batching adaptor.  Encoders and decoders attached to a batch queue
 * every packet and data delivery they produce instead of calling their handlers.  Protocol state (windows, rates,
 * counters, missing / pending sets, acks) advances immediately -- the reference's control flow
 * never depends on payload bytes -- while each GF region result is kept as a linear expression
 * over the payloads it came from.  ntc_batch_flush evaluates every pending expression with one
 * GPU launch per dependency level (payloads resident on the device), then calls the queued
 * handlers in production order (a queued packet as one prepare_packet call followed by
 * send_packet).  Each object's callback sequence is byte-for-byte the unbatched one
 * (encoder.hh:255-333, decoder.hh:88-300 semantics); only the time of some callbacks moves to the
 * flush.  Eager mode (ntc_batch_set_eager, off by default) emits an event that needs no GF result
 * (a source packet, a received source's delivery, an ack) of an object with nothing queued at
 * once, inside the call that produced it: callbacks then run both there and at the flush, so a
 * handler must be re-entrant with respect to the objects of the same batch.  Events that handlers
 * produce during a flush (e.g. a decoder fed from an encoder's packet handler) are queued for the
 * next flush: flush until ntc_batch_pending is 0 to drain such chains.  Asynchronous mode
 * (ntc_batch_set_async, off by default): ntc_batch_flush first delivers the events of the
 * previous flush, then starts the device work of the queued ones and returns without waiting;
 * those are delivered by the next ntc_batch_flush, so one flush's GPU round trip overlaps the
 * caller's work until the next (ntc_batch_pending counts them; flush until it is 0 to drain).
 * Each object's callback sequence is unchanged; objects with events in flight queue new ones
 * behind them.  Attaching an object to another batch or to NULL drains its current batch first.
 * Deleting an attached object discards its queued events; deleting a batch discards every queued
 * event and detaches its objects.  Memory: with a device present, data, packet and payload buffers
 * are pinned host blocks from a process-wide pool that keeps its peak size (the device reads new
 * payloads and writes results there directly; the pages sit on the calling CPU's NUMA node);
 * NTC_BATCH_UNPINNED=1 selects malloc'd buffers. */
typedef struct ntc_batch_t ntc_batch_t;
ntc_batch_t* ntc_new_batch(void) NTC_C_NOEXCEPT;
void ntc_delete_batch(ntc_batch_t* batch) NTC_C_NOEXCEPT;   /* NULL is a no-op */
void ntc_encoder_set_batch(ntc_encoder_t* enc, ntc_batch_t* batch, ntc_error* error) NTC_C_NOEXCEPT;
void ntc_decoder_set_batch(ntc_decoder_t* dec, ntc_batch_t* batch, ntc_error* error) NTC_C_NOEXCEPT;
void ntc_batch_flush(ntc_batch_t* batch, ntc_error* error) NTC_C_NOEXCEPT NTC_C_NONNULL;
size_t ntc_batch_pending(const ntc_batch_t* batch) NTC_C_NOEXCEPT NTC_C_NONNULL;
void ntc_batch_set_eager(ntc_batch_t* batch, int on) NTC_C_NOEXCEPT;   /* NULL is a no-op */
void ntc_batch_set_async(ntc_batch_t* batch, int on) NTC_C_NOEXCEPT;   /* NULL is a no-op */

/* GF(2^w) region work on host buffers, run on the MI355X engine (one H2D, one combine launch,
 * one D2H): the region operations of the C++ detail layer (include/netcode/detail/galois_field.hh,
 * encoder.hh, decoder.hh -- the reference's galois_field::multiply / multiply_add call sites,
 * galois_field.hh:65-92, detail/encoder.cc:35-57, detail/decoder.cc:173, 407, 524-532).
 *   ntc_gf_combine_host:      out[0..out_len) = sum_i coefs[i] * in_i, each input read over
 *                             lens[i] bytes and zero-extended; add = 1 XORs the sum into out.
 *   ntc_gf_combine_rows_host: rows outputs from the same inputs, out_s = sum_i coefs[i * rows + s]
 *                             * in_i (full decoding's M^-1 application).
 * w in {4, 8, 16, 32}; lengths <= 65535.  Return 0, or -1 with error set (no device, bad w). */
int ntc_gf_combine_host(uint32_t w, size_t n, const char* const* in, const uint16_t* lens,
                        const uint32_t* coefs, size_t out_len, char* out, int add,
                        ntc_error* error) NTC_C_NOEXCEPT;
int ntc_gf_combine_rows_host(uint32_t w, size_t n, const char* const* in, const uint16_t* lens,
                             size_t rows, const uint32_t* coefs, size_t out_len, char* const* out,
                             ntc_error* error) NTC_C_NOEXCEPT;

/* ntc::decoder::maybe_ack (reference decoder.hh:231-248): send an ack if the received-packet
 * threshold or the ack period has been reached. */
void ntc_decoder_maybe_ack(ntc_decoder_t* dec, ntc_error* error) NTC_C_NOEXCEPT NTC_C_NONNULL;

#ifdef __cplusplus
}
#endif
#endif
