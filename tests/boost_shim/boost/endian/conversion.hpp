// Tests-only stand-in for Boost.Endian (absent from the image): the one conversion the
// reference's tests/netcode/detail/test_packetizer.cc uses (lines 167-220) to craft truncated
// packets by hand.  Force-included (-include) into the reference test suite build, which gets it
// transitively from the reference's own packetizer.hh; no product code includes it.
#pragma once
#include <cstdint>

namespace boost {
namespace endian {

inline std::uint16_t native_to_big(std::uint16_t x) noexcept
{
  return static_cast<std::uint16_t>((x >> 8) | (x << 8));   // x86-64 / aarch64 hosts: little endian
}

inline std::uint16_t big_to_native(std::uint16_t x) noexcept { return native_to_big(x); }

}  // namespace endian
}  // namespace boost
