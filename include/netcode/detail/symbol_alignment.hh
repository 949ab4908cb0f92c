// netcode/detail/symbol_alignment.hh -- where a symbol starts inside a packet buffer
// (reference netcode/detail/symbol_alignment.hh:9-13).  Source and repair packets begin with a
// 7-byte header (type u8, id u32, symbol length u16); a packet reserves 16 - 7 = 9 bytes before
// its first byte so that the symbol behind the header starts 16-byte aligned and can be reduced
// in place.
#pragma once

#include <cstddef>

namespace ntc {
namespace detail {

constexpr std::size_t symbol_alignment = 16;
constexpr std::size_t source_and_repair_headers = 7;
static_assert(source_and_repair_headers <= symbol_alignment, "header longer than the alignment");

}  // namespace detail
}  // namespace ntc
