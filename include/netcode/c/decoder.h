/* netcode/c/decoder.h -- receiver side (reference netcode/c/decoder.h:28-94; semantics of
 * ntc::decoder, netcode/decoder.hh).  Region work runs on the MI355X engine (libntc_gf256). */
#ifndef NETCODE_C_DECODER_H
#define NETCODE_C_DECODER_H
#include "netcode/c/handlers.h"
#include "netcode/c/packet.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_decoder_t ntc_decoder_t;
typedef enum { ntc_in_order_yes, ntc_in_order_no } ntc_ordering_type;

ntc_decoder_t* ntc_new_decoder(uint8_t galois_field_size, ntc_ordering_type order,
                               ntc_packet_handler packet_handler, ntc_data_handler data_handler)
               NTC_C_NOEXCEPT;
void   ntc_delete_decoder(ntc_decoder_t* dec) NTC_C_NOEXCEPT;   /* NULL is a no-op */
/* Consumes `packet` (a source or a repair); returns the number of bytes read. */
size_t ntc_decoder_add_packet(ntc_decoder_t* dec, ntc_packet_t* packet, ntc_error* error)
       NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_decoder_generate_ack(ntc_decoder_t* dec, ntc_error* error) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_decoder_set_ack_period(ntc_decoder_t* dec, size_t period_ms) NTC_C_NOEXCEPT NTC_C_NONNULL;
void   ntc_decoder_set_ack_nb_packets(ntc_decoder_t* dec, uint16_t nb) NTC_C_NOEXCEPT NTC_C_NONNULL;

#ifdef __cplusplus
}
#endif
#endif
