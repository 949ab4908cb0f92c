// netcode/detail/source_list.hh -- the encoder's window (reference netcode/detail/
// source_list.hh:14-98): sources in insertion order (= ascending id), removable by sorted id
// lists (acks) or from the front (a full window).
#pragma once

#include <cstddef>
#include <cstdint>
#include <list>
#include <utility>

#include "netcode/detail/source.hh"
#include "netcode/detail/source_id_list.hh"

namespace ntc {
namespace detail {

class source_list final
{
public:
  using const_iterator = std::list<encoder_source>::const_iterator;

  const encoder_source& emplace(std::uint32_t id, byte_buffer&& symbol)
  {
    window_.emplace_back(id, std::move(symbol));
    return window_.back();
  }

  /// Remove every source whose id is in the sorted range [first, last): one merge-like pass over
  /// two ascending sequences.
  void erase(source_id_list::const_iterator first, source_id_list::const_iterator last) noexcept
  {
    auto it = window_.begin();
    while (it != window_.end() && first != last) {
      if (it->id() < *first) ++it;
      else if (*first < it->id()) ++first;
      else {
        it = window_.erase(it);
        ++first;
      }
    }
  }

  void pop_front() noexcept { window_.pop_front(); }
  std::size_t size() const noexcept { return window_.size(); }
  const_iterator cbegin() const noexcept { return window_.cbegin(); }
  const_iterator cend() const noexcept { return window_.cend(); }
  const_iterator begin() const noexcept { return window_.cbegin(); }
  const_iterator end() const noexcept { return window_.cend(); }

private:
  std::list<encoder_source> window_;
};

}  // namespace detail
}  // namespace ntc
