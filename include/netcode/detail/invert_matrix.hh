// netcode/detail/invert_matrix.hh -- ntc::detail::invert (reference netcode/detail/
// invert_matrix.{hh,cc}: invert_matrix.cc:9-128, jerasure's Gauss-Jordan order).
//
// The elimination walks STORAGE rows (square_matrix is column-major, so a storage row is a matrix
// column): swap in the first lower storage row with a non-zero pivot, scale by the pivot's
// inverse, clear the pivot column below, then back-substitute upwards.  On a singular matrix the
// result holds the failing index, which for this algorithm is always dimension - 1 (the reference
// decoder relies on it: detail/decoder.cc:448-468 drops its newest repair).  A default (empty)
// result means "inverted".  Scalar host arithmetic on at most 255 x 255 entries; the batched device
// inversion for whole generations is ntc_gf256_decode_batch / ntc_gf256_dense_invert_batch.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>

#include "netcode/detail/galois_field.hh"
#include "netcode/detail/square_matrix.hh"

namespace ntc {
namespace detail {

/// What invert() returns: empty (false) on success, the failing index otherwise (the shape of
/// the reference's boost::optional<std::size_t>).
class invert_failure
{
public:
  invert_failure() noexcept = default;
  explicit invert_failure(std::size_t index) noexcept : failed_{true}, index_{index} {}
  explicit operator bool() const noexcept { return failed_; }
  bool operator!() const noexcept { return !failed_; }
  std::size_t operator*() const noexcept { return index_; }
  std::size_t value() const noexcept { return index_; }

private:
  bool failed_ = false;
  std::size_t index_ = 0;
};

/// inv = mat^-1 over gf; mat is destroyed.  @return empty on success, else the failing index.
inline invert_failure invert(galois_field& gf, square_matrix& mat, square_matrix& inv) noexcept
{
  const std::size_t n = mat.dimension();
  for (std::size_t k = 0; k < n * n; ++k) inv[k] = (k % (n + 1) == 0) ? 1u : 0u;   // identity
  auto at = [n](square_matrix& m, std::size_t srow, std::size_t j) -> std::uint32_t& {
    return m[srow * n + j];                      // storage row srow, element j
  };
  for (std::size_t i = 0; i < n; ++i) {
    if (at(mat, i, i) == 0) {
      std::size_t swap_with = i + 1;
      while (swap_with < n && at(mat, swap_with, i) == 0) ++swap_with;
      if (swap_with == n) return invert_failure{n - 1};
      for (std::size_t j = 0; j < n; ++j) {
        std::swap(at(mat, i, j), at(mat, swap_with, j));
        std::swap(at(inv, i, j), at(inv, swap_with, j));
      }
    }
    const std::uint32_t pivot = at(mat, i, i);
    if (pivot != 1) {
      const std::uint32_t scale = gf.invert(pivot);
      for (std::size_t j = 0; j < n; ++j) {
        at(mat, i, j) = gf.multiply(at(mat, i, j), scale);
        at(inv, i, j) = gf.multiply(at(inv, i, j), scale);
      }
    }
    for (std::size_t r = i + 1; r < n; ++r) {
      const std::uint32_t f = at(mat, r, i);
      if (f == 0) continue;
      for (std::size_t j = 0; j < n; ++j) {
        at(mat, r, j) ^= f == 1 ? at(mat, i, j) : gf.multiply(f, at(mat, i, j));
        at(inv, r, j) ^= f == 1 ? at(inv, i, j) : gf.multiply(f, at(inv, i, j));
      }
    }
  }
  for (std::size_t i = n; i-- > 1;) {            // back substitution, bottom storage row first
    for (std::size_t r = 0; r < i; ++r) {
      const std::uint32_t f = at(mat, r, i);
      if (f == 0) continue;
      at(mat, r, i) = 0;
      for (std::size_t j = 0; j < n; ++j) at(inv, r, j) ^= gf.multiply(f, at(inv, i, j));
    }
  }
  return invert_failure{};
}

}  // namespace detail
}  // namespace ntc
