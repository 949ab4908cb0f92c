/* netcode/c/common.h -- shared macros of the netcode C ABI (MI355X build). */
#ifndef NETCODE_C_COMMON_H
#define NETCODE_C_COMMON_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
#define NTC_C_NOEXCEPT noexcept
#else
#include <stdbool.h>
#define NTC_C_NOEXCEPT
#endif
#define NTC_C_NONNULL __attribute__((nonnull))
#endif
