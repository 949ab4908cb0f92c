// netcode/detail/buffer.hh -- the byte containers of the reference's detail layer
// (reference netcode/detail/buffer.hh:66-82): 16-byte aligned vectors, so symbols can be read
// with wide loads.
//   byte_buffer       elements default-initialised on growth (no zeroing: data / packets)
//   zero_byte_buffer  elements value-initialised (zero) on growth (repair symbols, which are
//                     zero-padded to the longest source, detail/encoder.cc:26, 44-48)
#pragma once

#include <cstddef>
#include <new>
#include <utility>
#include <vector>

#include "netcode/detail/aligned_allocator.hh"

namespace ntc {
namespace detail {

// aligned_allocator whose argument-less construct() default-initialises (leaves a char
// uninitialised) instead of value-initialising: resize() of a large symbol costs no memset.
template <typename T>
struct uninit_aligned_allocator : aligned_allocator<T>
{
  template <typename U> struct rebind { using other = uninit_aligned_allocator<U>; };
  uninit_aligned_allocator() noexcept {}
  template <typename U> uninit_aligned_allocator(const uninit_aligned_allocator<U>&) noexcept {}

  template <typename U> void construct(U* p) { ::new (static_cast<void*>(p)) U; }
  template <typename U, typename A0, typename... As>
  void construct(U* p, A0&& a0, As&&... as)
  {
    ::new (static_cast<void*>(p)) U(std::forward<A0>(a0), std::forward<As>(as)...);
  }
};

template <typename T, typename U>
bool operator==(const uninit_aligned_allocator<T>&, const uninit_aligned_allocator<U>&) noexcept { return true; }
template <typename T, typename U>
bool operator!=(const uninit_aligned_allocator<T>&, const uninit_aligned_allocator<U>&) noexcept { return false; }

template <typename T>
using buffer = std::vector<T, uninit_aligned_allocator<T>>;

using byte_buffer = buffer<char>;
using zero_byte_buffer = std::vector<char, aligned_allocator<char>>;

}  // namespace detail
}  // namespace ntc
