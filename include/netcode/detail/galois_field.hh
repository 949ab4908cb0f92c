// netcode/detail/galois_field.hh -- ntc::detail::galois_field (reference
// netcode/detail/galois_field.hh:18-167) for w in {4, 8, 16, 32}, gf-complete's default fields.
// Scalar operations (coefficient, multiply, invert, multiply_size) are the engine's host helpers
// (netcode/gpu.h, libntc_gf256.so); region operations (multiply, multiply_add) run on the MI355X
// engine through libntc.so (ntc_gf_combine_host) -- there is no CPU region arithmetic here.
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

#include "netcode/c/ext.h"
#include "netcode/gpu.h"

namespace ntc {
namespace detail {

class galois_field final
{
public:
  galois_field(const galois_field&) = delete;
  galois_field& operator=(const galois_field&) = delete;
  galois_field(galois_field&&) = delete;
  galois_field& operator=(galois_field&&) = delete;

  /// @throw std::invalid_argument unless w is 4, 8, 16 or 32 (galois_field.hh:35-44).
  explicit galois_field(std::uint8_t w) : w_{w}
  {
    if (w != 4 && w != 8 && w != 16 && w != 32)
      throw std::invalid_argument("galois field size must be 4, 8, 16 or 32");
  }

  std::uint8_t size() const noexcept { return w_; }

  /// dst[0..len) = coeff * src[0..len)  (galois_field.hh:65-75)
  void multiply(const char* src, char* dst, std::size_t len, std::uint32_t coeff) { region(src, dst, len, coeff, 0); }

  /// dst[0..len) ^= coeff * src[0..len)  (galois_field.hh:83-92)
  void multiply_add(const char* src, char* dst, std::size_t len, std::uint32_t coeff) { region(src, dst, len, coeff, 1); }

  /// A u16 symbol size times coeff: bytewise for w <= 8, a field product for w = 16, the
  /// truncated product for w = 32 (galois_field.hh:96-120).
  std::uint16_t multiply_size(std::uint16_t size, std::uint32_t coeff) const noexcept
  {
    return ntc_gf_multiply_size(w_, size, coeff);
  }

  std::uint32_t multiply(std::uint32_t x, std::uint32_t y) const noexcept { return ntc_gf_multiply(w_, x, y); }
  std::uint32_t invert(std::uint32_t x) const noexcept { return ntc_gf_invert(w_, x); }

  /// The reference coefficient schedule (galois_field.hh:143-158, u32 wraparound).
  std::uint32_t coefficient(std::uint32_t repair_id, std::uint32_t src_id) const noexcept
  {
    return ntc_gf_coefficient(w_, repair_id, src_id);
  }

private:
  // Regions longer than the engine's u16 symbol bound go in 65535-byte pieces (w <= 32: every
  // piece boundary is a whole number of field elements, 65535 = 3 * 5 * 17 * 257 is odd, so use
  // 65532, a multiple of 4).
  void region(const char* src, char* dst, std::size_t len, std::uint32_t coeff, int add)
  {
    constexpr std::size_t kPiece = 65532;
    for (std::size_t off = 0; off < len; off += kPiece) {
      const std::size_t n = len - off < kPiece ? len - off : kPiece;
      const char* in = src + off;
      const std::uint16_t l = static_cast<std::uint16_t>(n);
      ntc_error e{ntc_no_error, nullptr};
      if (ntc_gf_combine_host(w_, 1, &in, &l, &coeff, n, dst + off, add, &e) != 0)
        throw std::runtime_error(std::string("galois_field region operation: ") +
                                 (e.message ? e.message : "MI355X engine unavailable"));
    }
  }

  const std::uint8_t w_;
};

}  // namespace detail
}  // namespace ntc
