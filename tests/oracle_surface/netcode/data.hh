// tests/oracle_surface (tests only): ntc::data (reference data.hh) -- a user payload.
#pragma once

#include "netcode/detail/buffer.hh"

namespace ntc {
using data = detail::byte_buffer;
}  // namespace ntc
