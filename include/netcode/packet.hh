// netcode/packet.hh -- a network packet (reference netcode/packet.hh:26-342).
// Vector-like byte container with the reference's member set and buffer layout: the bytes live in
// a 16-byte aligned detail::byte_buffer behind a 9-byte pre-pad, so in a source or repair packet
// the symbol after the 7-byte header starts 16-byte aligned (symbol() = data() + 7), and a packet
// built from a bare symbol buffer puts it exactly there.
#pragma once

#include <algorithm>
#include <cstddef>
#include <initializer_list>
#include <iterator>

#include "netcode/detail/buffer.hh"
#include "netcode/detail/symbol_alignment.hh"

namespace ntc {

namespace detail { struct serialize_packet; }

class packet final
{
  using buffer_type = detail::byte_buffer;

public:
  /// Bytes before the symbol; bytes before the packet's first byte.
  static constexpr std::size_t alignment = detail::symbol_alignment;
  static constexpr std::size_t shift = detail::symbol_alignment - detail::source_and_repair_headers;

  using value_type = buffer_type::value_type;
  using size_type = buffer_type::size_type;
  using difference_type = buffer_type::difference_type;
  using pointer = buffer_type::pointer;
  using const_pointer = buffer_type::const_pointer;
  using reference = buffer_type::reference;
  using const_reference = buffer_type::const_reference;
  using iterator = buffer_type::iterator;
  using const_iterator = buffer_type::const_iterator;

  packet() : m_buf(shift) {}
  packet(const packet&) = default;
  packet& operator=(const packet&) = default;
  packet(packet&&) = default;
  packet& operator=(packet&&) = default;

  /// @p size bytes, uninitialised.
  explicit packet(size_type size) : m_buf(shift + size) {}
  packet(size_type count, char value) : m_buf(shift + count, value) {}
  template <typename InputIterator>
  packet(InputIterator first, InputIterator last) : m_buf(shift)
  {
    m_buf.insert(m_buf.end(), first, last);
  }
  packet(std::initializer_list<char> init) : packet(init.begin(), init.end()) {}

  /// A packet whose symbol (at data() + 7) holds @p symbol; the 7 header bytes are unspecified.
  packet(const detail::byte_buffer& symbol) : m_buf(alignment + symbol.size())
  {
    std::copy(symbol.begin(), symbol.end(), m_buf.begin() + alignment);
  }
  packet(const detail::zero_byte_buffer& symbol) : m_buf(alignment + symbol.size())
  {
    std::copy(symbol.begin(), symbol.end(), m_buf.begin() + alignment);
  }

  void assign(size_type count, char value)
  {
    m_buf.resize(shift);
    m_buf.resize(shift + count, value);
  }
  template <typename InputIterator>
  void assign(InputIterator first, InputIterator last)
  {
    m_buf.resize(shift);
    m_buf.insert(m_buf.end(), first, last);
  }
  void assign(std::initializer_list<char> init) { assign(init.begin(), init.end()); }

  reference operator[](size_type pos) noexcept { return m_buf[shift + pos]; }
  const_reference operator[](size_type pos) const noexcept { return m_buf[shift + pos]; }
  char* data() noexcept { return m_buf.data() + shift; }
  const char* data() const noexcept { return m_buf.data() + shift; }

  iterator begin() noexcept { return m_buf.begin() + shift; }
  const_iterator begin() const noexcept { return m_buf.begin() + shift; }
  const_iterator cbegin() const noexcept { return m_buf.cbegin() + shift; }
  iterator end() noexcept { return m_buf.end(); }
  const_iterator end() const noexcept { return m_buf.end(); }
  const_iterator cend() const noexcept { return m_buf.cend(); }

  bool empty() const noexcept { return m_buf.size() == shift; }
  size_type size() const noexcept { return m_buf.size() - shift; }
  void reserve(size_type new_cap) { m_buf.reserve(shift + new_cap); }
  size_type capacity() const noexcept { return m_buf.capacity() - shift; }
  void shrink_to_fit() { m_buf.shrink_to_fit(); }
  void clear() { m_buf.resize(shift); }
  void push_back(char value) { m_buf.push_back(value); }
  void resize(size_type count) { m_buf.resize(shift + count); }
  void resize(size_type count, char value) { m_buf.resize(shift + count, value); }

  /// The symbol of a source or repair packet: 16-byte aligned, 7 bytes after data().
  char* symbol() noexcept { return m_buf.data() + alignment; }
  const char* symbol() const noexcept { return m_buf.data() + alignment; }

  friend bool operator==(const packet& a, const packet& b)
  {
    return a.size() == b.size() && std::equal(a.begin(), a.end(), b.begin());
  }
  friend bool operator!=(const packet& a, const packet& b) { return !(a == b); }

private:
  friend struct detail::serialize_packet;
  buffer_type m_buf;
};

}  // namespace ntc
