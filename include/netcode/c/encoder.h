/* netcode/c/encoder.h -- sender side (reference netcode/c/encoder.h:29-148; semantics of
 * ntc::encoder, netcode/encoder.hh).  Repairs are built by the MI355X engine (libntc_gf256). */
#ifndef NETCODE_C_ENCODER_H
#define NETCODE_C_ENCODER_H
#include "netcode/c/data.h"
#include "netcode/c/handlers.h"
#include "netcode/c/packet.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_encoder_t ntc_encoder_t;
typedef enum { ntc_systematic_yes, ntc_systematic_no } ntc_code_type;

/* galois_field_size: 4, 8, 16 or 32; NULL on OOM, unsupported size or no MI355X engine. */
ntc_encoder_t* ntc_new_encoder(uint8_t galois_field_size, ntc_packet_handler handler) NTC_C_NOEXCEPT;
void   ntc_delete_encoder(ntc_encoder_t* enc) NTC_C_NOEXCEPT;   /* NULL is a no-op */
/* Consumes `data` (left empty: resize or delete it afterwards). */
void   ntc_encoder_add_data(ntc_encoder_t* enc, ntc_data_t* data, ntc_error* error)
       NTC_C_NOEXCEPT NTC_C_NONNULL;
/* Gives an ack to the encoder; consumes `packet`; returns the number of bytes read. */
size_t ntc_encoder_add_packet(ntc_encoder_t* enc, ntc_packet_t* packet, ntc_error* error)
       NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_encoder_generate_repair(ntc_encoder_t* enc, ntc_error* error) NTC_C_NOEXCEPT NTC_C_NONNULL;
size_t ntc_encoder_window(ntc_encoder_t* enc) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_encoder_set_code_type(ntc_encoder_t* enc, ntc_code_type code_type) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_encoder_set_rate(ntc_encoder_t* enc, size_t rate) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_encoder_set_window_size(ntc_encoder_t* enc, size_t size) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_encoder_set_adaptive(ntc_encoder_t* enc, bool adaptive) NTC_C_NOEXCEPT NTC_C_NONNULL;

#ifdef __cplusplus
}
#endif
#endif
