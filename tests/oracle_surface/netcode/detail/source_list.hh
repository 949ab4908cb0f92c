// tests/oracle_surface (tests only): the encoder's window of sources, in id order (reference
// detail/source_list.hh).
#pragma once

#include <cstddef>
#include <cstdint>
#include <list>
#include <utility>

#include "netcode/detail/buffer.hh"
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
    l_.emplace_back(id, std::move(symbol));
    return l_.back();
  }

  // drop the sources whose ids the (sorted) range names; both sequences ascend
  void erase(source_id_list::const_iterator it, source_id_list::const_iterator end) noexcept
  {
    for (auto s = l_.begin(); s != l_.end() && it != end;) {
      if (s->id() == *it) {
        s = l_.erase(s);
        ++it;
      } else if (s->id() > *it) {
        ++it;
      } else {
        ++s;
      }
    }
  }

  std::size_t size() const noexcept { return l_.size(); }
  const_iterator cbegin() const noexcept { return l_.cbegin(); }
  const_iterator cend() const noexcept { return l_.cend(); }
  void pop_front() noexcept { l_.pop_front(); }

private:
  std::list<encoder_source> l_;
};

}  // namespace detail
}  // namespace ntc
