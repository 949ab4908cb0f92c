// netcode/detail/aligned_allocator.hh -- 16-byte aligned allocator for the public C++ surface.
// The reference aligns every data/symbol buffer on 16 bytes (netcode/detail/buffer.hh:66-82,
// symbol_alignment.hh:9-13) so region operations can use wide loads; this build keeps the
// guarantee for ntc::data / ntc::packet (the bytes are copied into the engine's own buffers).
#pragma once

#include <cstddef>
#include <cstdlib>
#include <limits>
#include <new>

namespace ntc {
namespace detail {

template <typename T, std::size_t Align = 16>
struct aligned_allocator
{
  using value_type = T;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  template <typename U> struct rebind { using other = aligned_allocator<U, Align>; };

  aligned_allocator() noexcept {}
  template <typename U> aligned_allocator(const aligned_allocator<U, Align>&) noexcept {}

  T* allocate(std::size_t n)
  {
    if (n > std::numeric_limits<std::size_t>::max() / sizeof(T)) throw std::bad_alloc{};
    void* p = nullptr;
    const std::size_t bytes = (n * sizeof(T) + Align - 1) / Align * Align;
    if (::posix_memalign(&p, Align, bytes ? bytes : Align) != 0) throw std::bad_alloc{};
    return static_cast<T*>(p);
  }
  void deallocate(T* p, std::size_t) noexcept { std::free(p); }
};

template <typename T, typename U, std::size_t A>
bool operator==(const aligned_allocator<T, A>&, const aligned_allocator<U, A>&) noexcept { return true; }
template <typename T, typename U, std::size_t A>
bool operator!=(const aligned_allocator<T, A>&, const aligned_allocator<U, A>&) noexcept { return false; }

}  // namespace detail
}  // namespace ntc
