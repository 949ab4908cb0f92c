/* netcode/c/data.h -- application data buffers (reference netcode/c/data.h:30-85). */
#ifndef NETCODE_C_DATA_H
#define NETCODE_C_DATA_H
#include "netcode/c/error.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ntc_data_t ntc_data_t;

ntc_data_t* ntc_new_data(uint16_t size) NTC_C_NOEXCEPT;                  /* NULL on OOM */
ntc_data_t* ntc_new_data_from(const char* src, uint16_t size) NTC_C_NOEXCEPT NTC_C_NONNULL;
void        ntc_delete_data(ntc_data_t* data) NTC_C_NOEXCEPT;   /* NULL is a no-op */
char*       ntc_data_buffer(ntc_data_t* data) NTC_C_NOEXCEPT NTC_C_NONNULL;   /* 16-B aligned */
uint16_t    ntc_data_get_size(const ntc_data_t* data) NTC_C_NOEXCEPT NTC_C_NONNULL;
/* Bytes a resize adds are default-initialised, as in the reference (buffer.hh:66-73): their
 * contents are unspecified.  After ntc_encoder_add_data the object may hold the storage of the
 * source that left the encoder's window, so they can be an earlier payload's bytes: write every
 * byte you resize to. */
void        ntc_data_resize(ntc_data_t* data, uint16_t new_size, ntc_error* error)
            NTC_C_NOEXCEPT NTC_C_NONNULL;

#ifdef __cplusplus
}
#endif
#endif
