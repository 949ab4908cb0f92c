// netcode/detail/ack.hh -- an acknowledgement (reference netcode/detail/ack.hh:11-89): the source
// ids a decoder knows and how many packets it received since its previous ack.
#pragma once

#include <cstdint>
#include <utility>

#include "netcode/detail/source_id_list.hh"

namespace ntc {
namespace detail {

class ack final
{
public:
  ack() = default;
  ack(source_id_list&& ids, std::uint16_t nb_packets) : ids_{std::move(ids)}, nb_packets_{nb_packets} {}
  ack(ack&&) = default;
  ack& operator=(ack&&) = default;
  ack(const ack&) = delete;
  ack& operator=(const ack&) = delete;

  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  std::uint16_t nb_packets() const noexcept { return nb_packets_; }
  std::uint16_t& nb_packets() noexcept { return nb_packets_; }

  void reset() noexcept
  {
    ids_.clear();
    nb_packets_ = 0;
  }

private:
  source_id_list ids_;
  std::uint16_t nb_packets_ = 0;
};

}  // namespace detail
}  // namespace ntc
