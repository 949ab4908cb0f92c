// tests/oracle_surface (tests only): ntc::detail::decoder (reference detail/decoder.{hh,cc}) = the
// oracle's streaming decoder core (or_dcore: the same state machine or_decode_batch and the
// oracle's public decoder run).  The accessors return snapshots of the core's state taken at the
// call, shaped like the reference's containers (sources and repairs by id; each missing source with
// the ids of the repairs that encode it).
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "netcode/detail/galois_field.hh"
#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/repair.hh"
#include "netcode/detail/source.hh"
#include "netcode/in_order.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

class decoder final
{
public:
  using repairs_set_type = std::map<std::uint32_t, decoder_repair>;
  using sources_set_type = std::map<std::uint32_t, decoder_source>;
  using missing_sources_type = std::map<std::uint32_t, std::set<std::uint32_t>>;

  decoder(std::uint8_t galois_field_size, std::function<void(const decoder_source&)> callback, in_order order)
    : gf_{galois_field_size}, cb_{std::move(callback)},
      core_{or_dcore_new(galois_field_size, order == in_order::yes, &deliver, this)}
  {}
  ~decoder() { or_dcore_free(core_); }
  decoder(const decoder&) = delete;
  decoder& operator=(const decoder&) = delete;

  void operator()(decoder_source&& src)
  {
    or_dcore_add_source(core_, src.id(), bytes(src.symbol()), src.symbol_size());
    ex_.rethrow();
  }

  void operator()(decoder_repair&& r)
  {
    std::vector<std::uint32_t> ids(r.source_ids().begin(), r.source_ids().end());
    or_dcore_add_repair(core_, r.id(), ids.data(), ids.size(), r.encoded_size(), bytes(r.symbol()),
                        r.symbol_size());
    ex_.rethrow();
  }

  decoder_source create_source_from_repair(const decoder_repair& r)
  {
    const std::uint32_t sid = *r.source_ids().begin();
    // multiply_size of a u16 is a u16: the source fits in 65535 bytes
    std::vector<std::uint8_t> out(65536);
    const std::uint16_t n = or_dcore_create_source_from_repair(core_, r.id(), sid, r.encoded_size(),
                                                               bytes(r.symbol()), r.symbol_size(), out.data());
    decoder_source s{sid, packet(n + packet::alignment), n};
    std::memcpy(s.symbol(), out.data(), n);
    return s;
  }

  void remove_source_from_repair(const decoder_source& src, decoder_repair& r)
  {
    std::uint16_t esz = r.encoded_size();
    or_dcore_remove_source_from_repair(core_, src.id(), bytes(src.symbol()), src.symbol_size(), r.id(), &esz,
                                       reinterpret_cast<std::uint8_t*>(r.symbol()));
    r.encoded_size() = esz;
    r.source_ids().erase(src.id());
  }

  const repairs_set_type& repairs() const
  {
    reps_.clear();
    for (std::size_t i = 0, n = or_dcore_count(core_, 1); i < n; ++i) {
      const std::uint32_t* ids;
      std::size_t nids;
      std::uint16_t esz, symsz;
      const std::uint8_t* sym;
      const std::uint32_t id = or_dcore_repair(core_, i, &ids, &nids, &esz, &sym, &symsz);
      detail::zero_byte_buffer b(reinterpret_cast<const char*>(sym), reinterpret_cast<const char*>(sym) + symsz);
      reps_.emplace(id, decoder_repair{id, esz, source_id_list(ids, ids + nids), packet(b), symsz});
    }
    return reps_;
  }

  const sources_set_type& sources() const
  {
    srcs_.clear();
    for (std::size_t i = 0, n = or_dcore_count(core_, 0); i < n; ++i) {
      const std::uint8_t* data;
      std::uint16_t len;
      const std::uint32_t id = or_dcore_source(core_, i, &data, &len);
      decoder_source s{id, packet(len + packet::alignment), len};
      if (len) std::memcpy(s.symbol(), data, len);
      srcs_.emplace(id, std::move(s));
    }
    return srcs_;
  }

  const missing_sources_type& missing_sources() const
  {
    miss_.clear();
    for (std::size_t i = 0, n = or_dcore_count(core_, 2); i < n; ++i) {
      const std::uint32_t* rids;
      std::size_t nr;
      const std::uint32_t sid = or_dcore_missing(core_, i, &rids, &nr);
      miss_.emplace(sid, std::set<std::uint32_t>(rids, rids + nr));
    }
    return miss_;
  }

  std::size_t nb_decoded() const noexcept { return or_dcore_count(core_, 3); }
  std::size_t nb_failed_full_decodings() const noexcept { return or_dcore_count(core_, 4); }
  std::size_t nb_useless_repairs() const noexcept { return or_dcore_count(core_, 5); }

private:
  static const std::uint8_t* bytes(const char* p) { return reinterpret_cast<const std::uint8_t*>(p); }

  static void deliver(void* ctx, std::uint32_t id, const std::uint8_t* data, std::uint16_t len)
  {
    auto* d = static_cast<decoder*>(ctx);
    try {
      decoder_source s{id, packet(len + packet::alignment), len};
      if (len) std::memcpy(s.symbol(), data, len);
      d->cb_(s);
    } catch (...) {
      d->ex_.park();
    }
  }

  galois_field gf_;
  std::function<void(const decoder_source&)> cb_;
  or_dcore* core_;
  parked_exception ex_;
  mutable repairs_set_type reps_;
  mutable sources_set_type srcs_;
  mutable missing_sources_type miss_;
};

}  // namespace detail
}  // namespace ntc
