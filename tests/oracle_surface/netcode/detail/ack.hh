// tests/oracle_surface (tests only): an acknowledgement (reference detail/ack.hh).
#pragma once

#include <cstdint>
#include <utility>

#include "netcode/detail/source_id_list.hh"

namespace ntc {
namespace detail {

class ack final
{
public:
  ack(const ack&) = delete;
  ack& operator=(const ack&) = delete;
  ack(ack&&) = default;
  ack& operator=(ack&&) = default;

  ack() : nb_{0} {}
  explicit ack(source_id_list&& ids, std::uint16_t nb_packets) : ids_{std::move(ids)}, nb_{nb_packets} {}

  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  std::uint16_t nb_packets() const noexcept { return nb_; }
  std::uint16_t& nb_packets() noexcept { return nb_; }
  void reset() noexcept
  {
    ids_.clear();
    nb_ = 0;
  }

private:
  source_id_list ids_;
  std::uint16_t nb_;
};

}  // namespace detail
}  // namespace ntc
