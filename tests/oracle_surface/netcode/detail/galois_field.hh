// tests/oracle_surface (tests only): ntc::detail::galois_field (reference detail/galois_field.hh)
// over the oracle's GF(2^w) arithmetic, w in {4, 8, 16, 32} (or_fw_*: gf-complete's default
// polynomials, the reference's coefficient schedule and size coding).
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>

#include "netcode/detail/oracle_bind.hh"

namespace ntc {
namespace detail {

class galois_field final
{
public:
  explicit galois_field(std::uint8_t w) : w_{w}
  {
    if (w != 4 && w != 8 && w != 16 && w != 32) throw std::runtime_error("unsupported field size");
  }

  std::uint8_t size() const noexcept { return w_; }

  std::uint32_t coefficient(std::uint32_t repair_id, std::uint32_t src_id) const noexcept
  {
    return or_fw_coefficient(w_, repair_id, src_id);
  }
  std::uint32_t multiply(std::uint32_t x, std::uint32_t y) const noexcept { return or_fw_mul(w_, x, y); }
  std::uint32_t invert(std::uint32_t x) const noexcept { return or_fw_inv(w_, x); }
  std::uint16_t multiply_size(std::uint16_t size, std::uint32_t c) const noexcept
  {
    return or_fw_multiply_size(w_, size, c);
  }

  void multiply(const char* src, char* dst, std::size_t len, std::uint32_t c) const noexcept
  {
    or_fw_region(w_, reinterpret_cast<const std::uint8_t*>(src), reinterpret_cast<std::uint8_t*>(dst), len, c, 0);
  }
  void multiply_add(const char* src, char* dst, std::size_t len, std::uint32_t c) const noexcept
  {
    or_fw_region(w_, reinterpret_cast<const std::uint8_t*>(src), reinterpret_cast<std::uint8_t*>(dst), len, c, 1);
  }

private:
  std::uint8_t w_;
};

}  // namespace detail
}  // namespace ntc
