// tests/oracle_surface (tests only): packet type tag of byte 0 (reference detail/packet_type.hh).
#pragma once

#include <cstdint>

#include "netcode/errors.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

enum class packet_type : std::uint8_t { ack = 0, repair = 1, source = 2 };

inline packet_type get_packet_type(const packet& p)
{
  const auto ty = static_cast<std::uint8_t>(p.data()[0]);
  if (ty > 2) throw packet_type_error{p};
  return static_cast<packet_type>(ty);
}

}  // namespace detail
}  // namespace ntc
