// tests/oracle_surface (tests only): ntc::detail::encoder (reference detail/encoder.{hh,cc}) =
// the oracle's repair builder, or_build_repair.
#pragma once

#include <algorithm>
#include <cstdint>
#include <vector>

#include "netcode/detail/galois_field.hh"
#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/repair.hh"
#include "netcode/detail/source_list.hh"

namespace ntc {
namespace detail {

class encoder final
{
public:
  explicit encoder(std::uint8_t galois_field_size) : gf_{galois_field_size} {}

  void operator()(encoder_repair& repair, source_list& sources)
  {
    std::vector<std::uint32_t> ids;
    std::vector<const std::uint8_t*> syms;
    std::vector<std::uint16_t> lens;
    std::uint16_t longest = 0;
    for (auto it = sources.cbegin(); it != sources.cend(); ++it) {
      ids.push_back(it->id());
      syms.push_back(reinterpret_cast<const std::uint8_t*>(it->symbol().data()));
      lens.push_back(it->size());
      longest = std::max(longest, it->size());
      repair.source_ids().insert(repair.source_ids().end(), it->id());
    }
    repair.symbol().assign(longest, 0);
    std::uint16_t esz = 0;
    or_build_repair(gf_.size(), repair.id(), ids.size(), ids.data(), syms.data(), lens.data(),
                    reinterpret_cast<std::uint8_t*>(repair.symbol().data()), &esz);
    repair.encoded_size() = esz;
  }

private:
  galois_field gf_;
};

}  // namespace detail
}  // namespace ntc
