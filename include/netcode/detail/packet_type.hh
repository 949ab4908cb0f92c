// netcode/detail/packet_type.hh -- the first byte of every packet (reference netcode/detail/
// packet_type.hh:11-36): 0 ack, 1 repair, 2 source; anything else is a packet_type_error.
#pragma once

#include <cstdint>

#include "netcode/errors.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

enum class packet_type : std::uint8_t { ack = 0, repair = 1, source = 2 };

/// @throw packet_type_error for an unknown type byte.
inline packet_type get_packet_type(const packet& p)
{
  const std::uint8_t t = static_cast<std::uint8_t>(p.data()[0]);
  if (t > static_cast<std::uint8_t>(packet_type::source)) throw packet_type_error{p};
  return static_cast<packet_type>(t);
}

}  // namespace detail
}  // namespace ntc
