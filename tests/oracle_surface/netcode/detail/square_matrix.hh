// tests/oracle_surface (tests only): a column-major square matrix of field elements (reference
// detail/square_matrix.hh); or_invert works on this storage.
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace ntc {
namespace detail {

class square_matrix final
{
public:
  explicit square_matrix(std::size_t n) : n_{n}, v_(n * n) {}

  std::uint32_t operator()(std::size_t row, std::size_t col) const noexcept { return v_[col * n_ + row]; }
  std::uint32_t& operator()(std::size_t row, std::size_t col) noexcept { return v_[col * n_ + row]; }
  std::uint32_t operator[](std::size_t i) const noexcept { return v_[i]; }
  std::uint32_t& operator[](std::size_t i) noexcept { return v_[i]; }
  const std::uint32_t* column(std::size_t col) const noexcept { return v_.data() + col * n_; }
  std::uint32_t* column(std::size_t col) noexcept { return v_.data() + col * n_; }
  std::uint32_t* data() noexcept { return v_.data(); }
  void resize(std::size_t n)
  {
    v_.resize(n * n);
    n_ = n;
  }
  std::size_t dimension() const noexcept { return n_; }

private:
  std::size_t n_;
  std::vector<std::uint32_t> v_;
};

}  // namespace detail
}  // namespace ntc
