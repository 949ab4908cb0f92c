/* netcode/c/handlers.h -- user callbacks (reference netcode/c/handlers.h:17-73).
 * Callbacks run synchronously on the caller's thread, in order, inside ntc_* calls. */
#ifndef NETCODE_C_HANDLERS_H
#define NETCODE_C_HANDLERS_H
#include "netcode/c/common.h"
#ifdef __cplusplus
extern "C" {
#endif

/* Some bytes of the packet being built are ready (called one or more times per packet). */
typedef void (*ntc_prepare_packet)(void* context, const char* pkt, size_t sz);
/* The packet whose bytes were given by ntc_prepare_packet is complete. */
typedef void (*ntc_send_packet)(void* context);

typedef struct {
  void* context;
  ntc_prepare_packet prepare_packet;
  ntc_send_packet send_packet;
} ntc_packet_handler;

/* A source has been received or decoded; `data` is 16-byte aligned and valid during the call. */
typedef void (*ntc_read_data)(void* context, const char* data, size_t sz);

typedef struct {
  void* context;
  ntc_read_data read_data;
} ntc_data_handler;

#ifdef __cplusplus
}
#endif
#endif
