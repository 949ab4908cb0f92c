// tests/oracle_surface (tests only): symbol layout constants (reference detail/symbol_alignment.hh).
#pragma once

#include <cstddef>

namespace ntc {
namespace detail {

static constexpr std::size_t symbol_alignment = 16;          // a symbol starts 16-B aligned
static constexpr std::size_t source_and_repair_headers = 7;  // type u8 + id u32 + size u16

}  // namespace detail
}  // namespace ntc
