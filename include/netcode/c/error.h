/* netcode/c/error.h -- error reporting of the C ABI.
 * Same types as the reference's netcode/c/error.h:11-33. */
#ifndef NETCODE_C_ERROR_H
#define NETCODE_C_ERROR_H
#include "netcode/c/common.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  ntc_no_error,          /* no error to report */
  ntc_unknown_error,     /* an unknown error occurred (message may describe it) */
  ntc_no_memory,         /* allocation failed */
  ntc_packet_type_error, /* a packet of the wrong type was given (e.g. a repair to an encoder) */
  ntc_overflow_error     /* a malformed packet would have been read past its end */
} ntc_error_type;

typedef struct {
  ntc_error_type type;
  /* Set for ntc_unknown_error only; points to library-owned, NUL-terminated, thread-local
   * storage valid until the next failing call on the same thread.  Never freed by the caller. */
  char* message;
} ntc_error;

#ifdef __cplusplus
}
#endif
#endif
