// tests/oracle_surface (tests only): ntc::detail::invert (reference detail/invert_matrix.hh) =
// the oracle's jerasure-order Gauss-Jordan, or_invert, in the matrix's field.
#pragma once

#include <cstddef>
#include <ostream>

#include "netcode/detail/galois_field.hh"
#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/square_matrix.hh"

namespace ntc {
namespace detail {

// empty = inverted; otherwise the failing index (the reference returns boost::optional<size_t>)
class invert_result
{
public:
  invert_result() noexcept = default;
  explicit invert_result(std::size_t i) noexcept : failed_{true}, index_{i} {}
  explicit operator bool() const noexcept { return failed_; }
  bool operator!() const noexcept { return !failed_; }
  std::size_t operator*() const noexcept { return index_; }
  friend std::ostream& operator<<(std::ostream& os, const invert_result& r)
  {
    return r.failed_ ? os << "failed at " << r.index_ : os << "inverted";
  }

private:
  bool failed_ = false;
  std::size_t index_ = 0;
};

inline invert_result invert(galois_field& gf, square_matrix& mat, square_matrix& inv)
{
  inv.resize(mat.dimension());
  const int old = or_field();
  or_set_field(gf.size());
  const long fail = or_invert(mat.data(), inv.data(), mat.dimension());
  or_set_field(old);
  return fail < 0 ? invert_result{} : invert_result{static_cast<std::size_t>(fail)};
}

}  // namespace detail
}  // namespace ntc
