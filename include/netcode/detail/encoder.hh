// netcode/detail/encoder.hh -- ntc::detail::encoder, the repair builder (reference
// netcode/detail/encoder.{hh,cc}, encoder.cc:15-64):
//   symbol       = sum_i c(repair id, source id_i) * source_i, each source zero-extended to the
//                  longest one (the symbol's length);
//   encoded_size = XOR_i multiply_size(size_i, c_i), the sources' sizes coded the same way;
//   source_ids  += the window's ids.
// The whole window is ONE combine launch on the MI355X engine (ntc_gf_combine_host), instead of
// one gf-complete region call per source.
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#include "netcode/c/ext.h"
#include "netcode/detail/galois_field.hh"
#include "netcode/detail/repair.hh"
#include "netcode/detail/source.hh"
#include "netcode/detail/source_list.hh"

namespace ntc {
namespace detail {

class encoder final
{
public:
  explicit encoder(std::uint8_t galois_field_size) : gf_{galois_field_size} {}

  /// Build @p repair (whose id is set) over every source of @p sources (non-empty).
  void operator()(encoder_repair& repair, source_list& sources)
  {
    std::vector<const char*> in;
    std::vector<std::uint16_t> lens;
    std::vector<std::uint32_t> coefs;
    std::uint16_t longest = 0, coded = 0;
    for (auto it = sources.cbegin(); it != sources.cend(); ++it) {
      const std::uint32_t c = gf_.coefficient(repair.id(), it->id());
      in.push_back(it->symbol().data());
      lens.push_back(it->size());
      coefs.push_back(c);
      longest = std::max(longest, it->size());
      coded = static_cast<std::uint16_t>(coded ^ gf_.multiply_size(it->size(), c));
      repair.source_ids().insert(repair.source_ids().end(), it->id());
    }
    repair.symbol().resize(longest);
    repair.encoded_size() = coded;
    if (longest == 0) return;
    ntc_error e{ntc_no_error, nullptr};
    if (ntc_gf_combine_host(gf_.size(), in.size(), in.data(), lens.data(), coefs.data(), longest,
                            repair.symbol().data(), 0, &e) != 0)
      throw std::runtime_error(std::string("detail::encoder: ") +
                               (e.message ? e.message : "MI355X engine unavailable"));
  }

  galois_field& field() noexcept { return gf_; }

private:
  galois_field gf_;
};

}  // namespace detail
}  // namespace ntc
