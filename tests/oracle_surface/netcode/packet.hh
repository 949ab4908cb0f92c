// tests/oracle_surface (tests only): ntc::packet (reference packet.hh) -- wire bytes preceded by
// `shift` bytes of slack, so that a source's or repair's symbol (7 bytes into the packet) sits at
// a 16-byte boundary of the underlying buffer.
#pragma once

#include <algorithm>
#include <cstddef>
#include <initializer_list>
#include <iterator>
#include <type_traits>

#include "netcode/detail/buffer.hh"
#include "netcode/detail/symbol_alignment.hh"

namespace ntc {

class packet
{
public:
  static constexpr std::size_t alignment = detail::symbol_alignment;
  static constexpr std::size_t shift = detail::symbol_alignment - detail::source_and_repair_headers;

  using value_type = char;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  using pointer = char*;
  using const_pointer = const char*;
  using reference = char&;
  using const_reference = const char&;
  using iterator = detail::byte_buffer::iterator;
  using const_iterator = detail::byte_buffer::const_iterator;

  packet() : b_(shift) {}
  explicit packet(size_type n) : b_(n + shift) {}
  packet(size_type n, char v) : b_(n + shift, v) {}

  template <typename It, typename = typename std::iterator_traits<It>::iterator_category>
  packet(It first, It last) : b_(static_cast<size_type>(std::distance(first, last)) + shift)
  {
    std::copy(first, last, b_.begin() + shift);
  }

  packet(std::initializer_list<char> init) : packet(init.begin(), init.end()) {}

  // a bare symbol, placed at the aligned symbol offset
  packet(const detail::byte_buffer& sym) : b_(sym.size() + alignment)
  {
    std::copy(sym.begin(), sym.end(), b_.begin() + alignment);
  }
  packet(const detail::zero_byte_buffer& sym) : b_(sym.size() + alignment)
  {
    std::copy(sym.begin(), sym.end(), b_.begin() + alignment);
  }

  char* data() noexcept { return b_.data() + shift; }
  const char* data() const noexcept { return b_.data() + shift; }
  size_type size() const noexcept { return b_.size() - shift; }
  bool empty() const noexcept { return size() == 0; }

  iterator begin() noexcept { return b_.begin() + shift; }
  const_iterator begin() const noexcept { return b_.begin() + shift; }
  const_iterator cbegin() const noexcept { return b_.cbegin() + shift; }
  iterator end() noexcept { return b_.end(); }
  const_iterator end() const noexcept { return b_.end(); }
  const_iterator cend() const noexcept { return b_.cend(); }

  reference operator[](size_type i) noexcept { return b_[i + shift]; }
  const_reference operator[](size_type i) const noexcept { return b_[i + shift]; }

  void reserve(size_type n) { b_.reserve(n + shift); }
  size_type capacity() const noexcept { return b_.capacity() - shift; }
  void shrink_to_fit() { b_.shrink_to_fit(); }
  void clear() { b_.resize(shift); }
  void push_back(char c) { b_.push_back(c); }
  void resize(size_type n) { b_.resize(n + shift); }
  void resize(size_type n, char v) { b_.resize(n + shift, v); }
  void assign(size_type n, char v)
  {
    resize(n);
    std::fill(begin(), end(), v);
  }
  template <typename It, typename = typename std::iterator_traits<It>::iterator_category>
  void assign(It first, It last)
  {
    resize(static_cast<size_type>(std::distance(first, last)));
    std::copy(first, last, begin());
  }
  void assign(std::initializer_list<char> init) { assign(init.begin(), init.end()); }

  // the symbol of a source / repair packet (the first symbol copy, 7 bytes into the packet)
  char* symbol() noexcept { return b_.data() + alignment; }
  const char* symbol() const noexcept { return b_.data() + alignment; }

private:
  detail::byte_buffer b_;
};

}  // namespace ntc
