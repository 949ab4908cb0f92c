// netcode/detail/decoder.hh -- ntc::detail::decoder, the receiver state machine of the reference
// (netcode/detail/decoder.{hh,cc}), re-authored over std containers with every GF region
// operation on the MI355X engine (libntc.so ntc_gf_combine_host / _rows_host).
//
// Semantics reproduced (detail/decoder.cc line references):
//  * source arrival (:33-50): dropped when outdated (< the last repair's first id) or duplicate;
//    otherwise delivered (in order or not) and removed from every pending repair that encodes
//    it, which may leave single-unknown repairs that are peeled recursively (:249-337); then a
//    full decoding is attempted;
//  * repair arrival (:54-152): dropped when outdated or duplicate; older state is dropped
//    (:341-389); a repair whose sources are all known is useless (:79-89); known sources are
//    subtracted from it IN PLACE (its symbol inside its packet, :393-408), the others linked as
//    missing; one unknown left -> the source is rebuilt (:156-178), else full decoding;
//  * full decoding (:412-566) when #missing == #repairs: the coefficient matrix (column =
//    repair, row = missing source, both by ascending id) is inverted (detail::invert); a
//    singular one drops the repair at the failing index -- the newest -- and counts a failure;
//    otherwise every missing source = sum_q inv * repair_q over min(size, repair size) bytes, its
//    size from the encoded sizes the same way, then repairs and missing sources are cleared.
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <iterator>
#include <map>
#include <set>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "netcode/c/ext.h"
#include "netcode/detail/galois_field.hh"
#include "netcode/detail/invert_matrix.hh"
#include "netcode/detail/repair.hh"
#include "netcode/detail/source.hh"
#include "netcode/detail/square_matrix.hh"
#include "netcode/in_order.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

class decoder final
{
public:
  using repairs_set_type = std::map<std::uint32_t, decoder_repair>;
  using sources_set_type = std::map<std::uint32_t, decoder_source>;

private:
  struct by_repair_id
  {
    bool operator()(const repairs_set_type::iterator& a, const repairs_set_type::iterator& b) const noexcept
    {
      return a->first < b->first;
    }
  };

public:
  /// The repairs (by ascending id) that still encode a missing source.
  using repairs_iterators_type = std::set<repairs_set_type::iterator, by_repair_id>;
  using missing_sources_type = std::map<std::uint32_t, repairs_iterators_type>;

  decoder(std::uint8_t galois_field_size, std::function<void(const decoder_source&)> callback,
          in_order order)
    : gf_{galois_field_size}, in_order_{order == in_order::yes}, deliver_{std::move(callback)},
      coefficients_{32}, inverse_{32}
  {}

  decoder(const decoder&) = delete;
  decoder& operator=(const decoder&) = delete;

  /// A received source (:33-50).
  void operator()(decoder_source&& src)
  {
    if (has_last_id_ && src.id() < last_id_) return;        // outdated
    if (sources_.count(src.id())) return;                    // duplicate
    add_source_recursive(std::move(src));
    attempt_full_decoding();
  }

  /// A received repair (:54-152); its source id list must not be empty.
  void operator()(decoder_repair&& incoming)
  {
    if (incoming.source_ids().empty()) throw std::invalid_argument("repair without source ids");
    if (has_last_id_ && incoming.source_ids().back() < last_id_) return;   // outdated
    if (repairs_.count(incoming.id())) return;                              // duplicate
    drop_outdated(incoming.source_ids().front());
    const auto& ids = incoming.source_ids();
    if (std::all_of(ids.begin(), ids.end(), [this](std::uint32_t s) { return sources_.count(s) != 0; })) {
      ++nb_useless_;
      return;
    }
    const std::uint32_t rid = incoming.id();
    const auto r_it = repairs_.emplace(rid, std::move(incoming)).first;
    decoder_repair& r = r_it->second;

    // Split the ids into received sources (subtracted now, all in one engine launch) and missing
    // ones (linked to this repair), highest id first like the reference's walk.
    std::vector<std::uint32_t> known;
    for (auto it = r.source_ids().rbegin(); it != r.source_ids().rend(); ++it) {
      if (sources_.count(*it)) known.push_back(*it);
      else missing_[*it].insert(r_it);
    }
    subtract_sources(known, r);
    for (std::uint32_t id : known) r.source_ids().erase(id);

    if (r.source_ids().size() == 1) {
      decoder_source rebuilt = create_source_from_repair(r);
      missing_.erase(rebuilt.id());
      repairs_.erase(r_it);
      add_source_recursive(std::move(rebuilt));
      return;
    }
    attempt_full_decoding();
  }

  /// The source a single-source repair encodes (:156-178).
  decoder_source create_source_from_repair(const decoder_repair& r)
  {
    const std::uint32_t sid = r.source_ids().front();
    const std::uint32_t inv = gf_.invert(gf_.coefficient(r.id(), sid));
    const std::uint16_t size = gf_.multiply_size(r.encoded_size(), inv);
    decoder_source src{sid, packet(size + packet::alignment), size};
    gf_.multiply(r.symbol(), src.symbol(), size, inv);
    ++nb_decoded_;
    return src;
  }

  /// Subtract a known source from a repair and forget its id (:182-191).
  void remove_source_from_repair(const decoder_source& src, decoder_repair& r)
  {
    subtract(src, r);
    r.source_ids().erase(src.id());
  }

  const repairs_set_type& repairs() const noexcept { return repairs_; }
  const sources_set_type& sources() const noexcept { return sources_; }
  const missing_sources_type& missing_sources() const noexcept { return missing_; }
  std::size_t nb_useless_repairs() const noexcept { return nb_useless_; }
  std::size_t nb_failed_full_decodings() const noexcept { return nb_failed_; }
  std::size_t nb_decoded() const noexcept { return nb_decoded_; }

private:
  // r ^= c(r, src) * src and its encoded size likewise (:393-408): in place in r's packet.
  void subtract(const decoder_source& src, decoder_repair& r)
  {
    const std::uint32_t c = gf_.coefficient(r.id(), src.id());
    r.encoded_size() = static_cast<std::uint16_t>(gf_.multiply_size(src.symbol_size(), c) ^ r.encoded_size());
    gf_.multiply_add(src.symbol(), r.symbol(), src.symbol_size(), c);
  }

  // The same for several known sources of one repair, one launch (XOR order is irrelevant).
  void subtract_sources(const std::vector<std::uint32_t>& ids, decoder_repair& r)
  {
    if (ids.empty()) return;
    std::vector<const char*> in;
    std::vector<std::uint16_t> lens;
    std::vector<std::uint32_t> coefs;
    std::uint16_t longest = 0;
    for (std::uint32_t id : ids) {
      const decoder_source& s = sources_.at(id);
      const std::uint32_t c = gf_.coefficient(r.id(), id);
      r.encoded_size() = static_cast<std::uint16_t>(gf_.multiply_size(s.symbol_size(), c) ^ r.encoded_size());
      in.push_back(s.symbol());
      lens.push_back(s.symbol_size());
      coefs.push_back(c);
      longest = std::max(longest, s.symbol_size());
    }
    if (longest == 0) return;
    ntc_error e{ntc_no_error, nullptr};
    if (ntc_gf_combine_host(gf_.size(), in.size(), in.data(), lens.data(), coefs.data(), longest,
                            r.symbol(), 1, &e) != 0)
      throw std::runtime_error(std::string("detail::decoder: ") + (e.message ? e.message : "engine"));
  }

  void deliver_or_hold(const decoder_source& s)
  {
    if (!in_order_) {
      deliver_(s);
    } else if (s.id() == next_in_order_) {
      deliver_(s);
      ++next_in_order_;
      flush_ordered_sources();
    } else {
      held_.emplace(s.id(), &s);
    }
  }

  // :249-337
  void add_source_recursive(decoder_source&& src)
  {
    if (!in_order_) {
      deliver_(src);
    } else if (src.id() == next_in_order_) {
      deliver_(src);
      ++next_in_order_;
      flush_ordered_sources();
    }
    const auto m = missing_.find(src.id());
    if (m != missing_.end()) {
      for (const auto& r_it : m->second) remove_source_from_repair(src, r_it->second);
      missing_.erase(m);
    }
    // peel: a missing source referenced by exactly one repair that encodes only it
    for (auto it = missing_.begin(); it != missing_.end();) {
      if (it->second.size() == 1 && (*it->second.begin())->second.source_ids().size() == 1) {
        const auto r_it = *it->second.begin();
        decoder_source peeled = create_source_from_repair(r_it->second);
        repairs_.erase(r_it);
        it = missing_.erase(it);
        add_source_recursive(std::move(peeled));
      } else {
        ++it;
      }
    }
    const std::uint32_t id = src.id();
    const auto ins = sources_.emplace(id, std::move(src)).first;
    if (in_order_ && id > next_in_order_) held_.emplace(id, &ins->second);
  }

  // :341-389: everything older than `id` is outdated
  void drop_outdated(std::uint32_t id)
  {
    has_last_id_ = true;
    last_id_ = id;
    for (auto it = repairs_.begin(); it != repairs_.end();) {
      if (it->second.source_ids().front() < id) {
        for (std::uint32_t sid : it->second.source_ids()) {
          const auto m = missing_.find(sid);
          if (m != missing_.end()) m->second.erase(it);
        }
        it = repairs_.erase(it);
      } else {
        ++it;
      }
    }
    if (in_order_) {
      const auto stop = held_.lower_bound(id);
      for (auto it = held_.begin(); it != stop;) {
        deliver_(*it->second);
        it = held_.erase(it);
      }
      next_in_order_ = std::max(next_in_order_, id);
      flush_ordered_sources();
    }
    sources_.erase(sources_.begin(), sources_.lower_bound(id));
    missing_.erase(missing_.begin(), missing_.lower_bound(id));
  }

  // :412-566
  void attempt_full_decoding()
  {
    if (repairs_.empty() || missing_.empty() || missing_.size() > repairs_.size()) return;
    const std::size_t n = repairs_.size();
    coefficients_.resize(n);
    std::size_t col = 0;
    for (const auto& r : repairs_) {
      std::size_t row = 0;
      for (const auto& miss : missing_) {
        coefficients_(row, col) = r.second.source_ids().count(miss.first) ? gf_.coefficient(r.first, miss.first) : 0u;
        ++row;
      }
      ++col;
    }
    inverse_.resize(n);
    if (const invert_failure bad = invert(gf_, coefficients_, inverse_)) {
      ++nb_failed_;
      auto r_it = std::next(repairs_.begin(), static_cast<std::ptrdiff_t>(*bad));
      for (std::uint32_t sid : r_it->second.source_ids()) missing_[sid].erase(r_it);
      repairs_.erase(r_it);
      return;
    }

    // every missing source at once: out_s = sum_q inverse(q, s) * repair_q (one engine launch)
    std::vector<const decoder_repair*> reps;
    for (const auto& r : repairs_) reps.push_back(&r.second);
    std::vector<std::uint16_t> sizes(n, 0);
    std::vector<std::uint32_t> coefs(n * n);
    std::vector<const char*> in(n);
    std::vector<std::uint16_t> lens(n);
    std::uint16_t longest = 0;
    for (std::size_t s = 0; s < n; ++s) {
      for (std::size_t q = 0; q < n; ++q) {
        const std::uint32_t c = inverse_(q, s);
        coefs[q * n + s] = c;
        if (c) sizes[s] = static_cast<std::uint16_t>(gf_.multiply_size(reps[q]->encoded_size(), c) ^ sizes[s]);
      }
      longest = std::max(longest, sizes[s]);
    }
    for (std::size_t q = 0; q < n; ++q) {
      in[q] = reps[q]->symbol();
      lens[q] = reps[q]->symbol_size();
    }
    std::vector<packet> rebuilt;
    std::vector<char*> outs;
    rebuilt.reserve(n);
    for (std::size_t s = 0; s < n; ++s) {
      // zeroed, symbol at the packet's aligned slot (:503-505); at least `longest` bytes behind
      // symbol() so the launch can write every output over the same length
      rebuilt.emplace_back(longest + packet::alignment, 0);
      outs.push_back(rebuilt.back().symbol());
    }
    if (longest) {
      ntc_error e{ntc_no_error, nullptr};
      if (ntc_gf_combine_rows_host(gf_.size(), n, in.data(), lens.data(), n, coefs.data(), longest,
                                   outs.data(), &e) != 0)
        throw std::runtime_error(std::string("detail::decoder: ") + (e.message ? e.message : "engine"));
      for (std::size_t s = 0; s < n; ++s)    // bytes past a source's own size are not its data
        std::fill(outs[s] + sizes[s], outs[s] + longest, 0);
    }
    std::size_t s = 0;
    for (const auto& miss : missing_) {
      const auto ins = sources_.emplace(miss.first, decoder_source{miss.first, std::move(rebuilt[s]), sizes[s]}).first;
      deliver_or_hold(ins->second);
      ++s;
    }
    nb_decoded_ += missing_.size();
    repairs_.clear();
    missing_.clear();
  }

  // :570-591: deliver held sources that now follow the in-order cursor
  void flush_ordered_sources()
  {
    auto it = held_.find(next_in_order_);
    while (it != held_.end() && it->first == next_in_order_) {
      deliver_(*it->second);
      it = held_.erase(it);
      ++next_in_order_;
    }
  }

  galois_field gf_;
  const bool in_order_;
  std::uint32_t next_in_order_ = 0;
  std::map<std::uint32_t, const decoder_source*> held_;   // received out of order, not delivered
  const std::function<void(const decoder_source&)> deliver_;
  repairs_set_type repairs_;
  sources_set_type sources_;
  bool has_last_id_ = false;
  std::uint32_t last_id_ = 0;
  missing_sources_type missing_;
  std::size_t nb_useless_ = 0, nb_failed_ = 0, nb_decoded_ = 0;
  square_matrix coefficients_;
  square_matrix inverse_;
};

}  // namespace detail
}  // namespace ntc
