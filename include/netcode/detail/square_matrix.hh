// netcode/detail/square_matrix.hh -- n x n matrix of field elements stored column by column
// (reference netcode/detail/square_matrix.hh:12-97: (row, col) lives at col * n + row, and
// operator[] walks that storage directly -- detail::invert works on storage rows, which are the
// matrix's columns).
#pragma once

#include <cstddef>
#include <cstdint>

#include "netcode/detail/buffer.hh"

namespace ntc {
namespace detail {

class square_matrix final
{
public:
  explicit square_matrix(std::size_t n) : n_{n}, cells_(n * n) {}

  std::uint32_t operator()(std::size_t row, std::size_t col) const noexcept { return cells_[col * n_ + row]; }
  std::uint32_t& operator()(std::size_t row, std::size_t col) noexcept { return cells_[col * n_ + row]; }

  const std::uint32_t* column(std::size_t col) const noexcept { return cells_.data() + col * n_; }
  std::uint32_t* column(std::size_t col) noexcept { return cells_.data() + col * n_; }

  std::uint32_t operator[](std::size_t i) const noexcept { return cells_[i]; }
  std::uint32_t& operator[](std::size_t i) noexcept { return cells_[i]; }

  void resize(std::size_t n)
  {
    cells_.resize(n * n);
    n_ = n;
  }
  std::size_t dimension() const noexcept { return n_; }

private:
  std::size_t n_;
  buffer<std::uint32_t> cells_;
};

}  // namespace detail
}  // namespace ntc
