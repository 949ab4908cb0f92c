// netcode/data.hh -- application data (reference netcode/data.hh: ntc::data).
// A std::vector<char> with a 16-byte aligned allocator, like the reference's detail::byte_buffer.
#pragma once

#include <vector>

#include "netcode/detail/aligned_allocator.hh"

namespace ntc {

/// The type to hold application data.
using data = std::vector<char, detail::aligned_allocator<char>>;

}  // namespace ntc
