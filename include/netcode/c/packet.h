/* netcode/c/packet.h -- network packet buffers (reference netcode/c/packet.h:30-85).
 * Internally the payload starts 9 bytes into the allocation so that, after the 7-byte
 * source/repair header, a symbol is 16-byte aligned (reference packet.hh:30-36). */
#ifndef NETCODE_C_PACKET_H
#define NETCODE_C_PACKET_H
#include "netcode/c/error.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_packet_t ntc_packet_t;

ntc_packet_t* ntc_new_packet(uint16_t size) NTC_C_NOEXCEPT;              /* NULL on OOM */
ntc_packet_t* ntc_new_packet_from(const char* src, uint16_t size) NTC_C_NOEXCEPT NTC_C_NONNULL;
void          ntc_delete_packet(ntc_packet_t* packet) NTC_C_NOEXCEPT;   /* NULL is a no-op */
char*         ntc_packet_buffer(ntc_packet_t* packet) NTC_C_NOEXCEPT NTC_C_NONNULL;
uint16_t      ntc_packet_get_size(const ntc_packet_t* packet) NTC_C_NOEXCEPT NTC_C_NONNULL;
void          ntc_packet_resize(ntc_packet_t* packet, uint16_t new_size, ntc_error* error)
              NTC_C_NOEXCEPT NTC_C_NONNULL;

#ifdef __cplusplus
}
#endif
#endif
