// tests/oracle_surface (tests only): 16-byte aligned byte vectors (reference detail/buffer.hh):
// byte_buffer default-initialises on growth, zero_byte_buffer zero-fills.
#pragma once

#include <cstddef>
#include <cstdlib>
#include <new>
#include <utility>
#include <vector>

namespace ntc {
namespace detail {

template <typename T, bool Zero>
struct aligned16_allocator
{
  using value_type = T;
  template <typename U> struct rebind { using other = aligned16_allocator<U, Zero>; };

  aligned16_allocator() noexcept = default;
  template <typename U> aligned16_allocator(const aligned16_allocator<U, Zero>&) noexcept {}

  T* allocate(std::size_t n)
  {
    void* p = nullptr;
    if (posix_memalign(&p, 16, n ? n * sizeof(T) : 16) != 0) throw std::bad_alloc{};
    return static_cast<T*>(p);
  }
  void deallocate(T* p, std::size_t) noexcept { std::free(p); }

  template <typename U> void construct(U* p)
  {
    if (Zero) ::new (static_cast<void*>(p)) U();
    else ::new (static_cast<void*>(p)) U;
  }
  template <typename U, typename... A> void construct(U* p, A&&... a)
  {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }

  friend bool operator==(const aligned16_allocator&, const aligned16_allocator&) noexcept { return true; }
  friend bool operator!=(const aligned16_allocator&, const aligned16_allocator&) noexcept { return false; }
};

template <typename T> using buffer = std::vector<T, aligned16_allocator<T, false>>;
using byte_buffer = buffer<char>;
using zero_byte_buffer = std::vector<char, aligned16_allocator<char, true>>;

}  // namespace detail
}  // namespace ntc
