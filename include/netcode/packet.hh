// netcode/packet.hh -- a network packet (reference netcode/packet.hh:26-342).
// Vector-like byte container with the reference's member set.  The reference keeps a 9-byte
// pre-pad so a symbol after the 7-byte header is 16-B aligned; this build copies packets into the
// engine's own aligned buffers (libntc.so), so the public type only has to be a byte vector.
#pragma once

#include <cstddef>
#include <initializer_list>
#include <vector>

#include "netcode/detail/aligned_allocator.hh"

namespace ntc {

class packet final
{
  using buffer_type = std::vector<char, detail::aligned_allocator<char>>;

public:
  using value_type = buffer_type::value_type;
  using size_type = buffer_type::size_type;
  using difference_type = buffer_type::difference_type;
  using pointer = buffer_type::pointer;
  using const_pointer = buffer_type::const_pointer;
  using reference = buffer_type::reference;
  using const_reference = buffer_type::const_reference;
  using iterator = buffer_type::iterator;
  using const_iterator = buffer_type::const_iterator;

  packet() = default;
  packet(const packet&) = default;
  packet& operator=(const packet&) = default;
  packet(packet&&) = default;
  packet& operator=(packet&&) = default;

  explicit packet(size_type size) : m_buffer(size) {}
  packet(size_type count, char value) : m_buffer(count, value) {}
  template <typename InputIterator>
  packet(InputIterator first, InputIterator last) : m_buffer(first, last) {}
  packet(std::initializer_list<char> init) : m_buffer(init) {}

  void assign(size_type count, char value) { m_buffer.assign(count, value); }
  template <typename InputIterator>
  void assign(InputIterator first, InputIterator last) { m_buffer.assign(first, last); }
  void assign(std::initializer_list<char> init) { m_buffer.assign(init); }

  reference operator[](size_type pos) noexcept { return m_buffer[pos]; }
  const_reference operator[](size_type pos) const noexcept { return m_buffer[pos]; }
  char* data() noexcept { return m_buffer.data(); }
  const char* data() const noexcept { return m_buffer.data(); }

  iterator begin() noexcept { return m_buffer.begin(); }
  const_iterator begin() const noexcept { return m_buffer.begin(); }
  const_iterator cbegin() const noexcept { return m_buffer.cbegin(); }
  iterator end() noexcept { return m_buffer.end(); }
  const_iterator end() const noexcept { return m_buffer.end(); }
  const_iterator cend() const noexcept { return m_buffer.cend(); }

  bool empty() const noexcept { return m_buffer.empty(); }
  size_type size() const noexcept { return m_buffer.size(); }
  void reserve(size_type new_cap) { m_buffer.reserve(new_cap); }
  size_type capacity() const noexcept { return m_buffer.capacity(); }
  void shrink_to_fit() { m_buffer.shrink_to_fit(); }
  void clear() noexcept { m_buffer.clear(); }
  void push_back(char value) { m_buffer.push_back(value); }
  void resize(size_type count) { m_buffer.resize(count); }
  void resize(size_type count, char value) { m_buffer.resize(count, value); }

  /// The symbol of a source or repair packet (bytes after the 7-byte header).
  char* symbol() noexcept { return m_buffer.data() + 7; }
  const char* symbol() const noexcept { return m_buffer.data() + 7; }

  friend bool operator==(const packet& a, const packet& b) { return a.m_buffer == b.m_buffer; }
  friend bool operator!=(const packet& a, const packet& b) { return a.m_buffer != b.m_buffer; }

private:
  buffer_type m_buffer;
};

}  // namespace ntc
