// tests/oracle_surface (tests only): ntc::detail::packetizer (reference detail/packetizer.hh) =
// the oracle's wire format: or_write_{ack,repair,source}_packet and or_parse_packet.  Each packet
// goes to the handler as one piece followed by the end-of-packet call.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "netcode/detail/ack.hh"
#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/packet_type.hh"
#include "netcode/detail/repair.hh"
#include "netcode/detail/source.hh"
#include "netcode/detail/source_id_list.hh"
#include "netcode/errors.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

template <typename PacketHandler>
class packetizer final
{
public:
  explicit packetizer(PacketHandler& h) : h_(h) {}

  void write_ack(const ack& a)
  {
    std::vector<std::uint8_t> out(or_packet_bound(0, a.source_ids().size()));
    emit(out, or_write_ack_packet(a.nb_packets(), a.source_ids().data(), a.source_ids().size(), out.data()));
  }

  void write_repair(const encoder_repair& r)
  {
    std::vector<std::uint8_t> out(or_packet_bound(r.symbol().size(), r.source_ids().size()));
    emit(out, or_write_repair_packet(r.id(), reinterpret_cast<const std::uint8_t*>(r.symbol().data()),
                                     static_cast<std::uint16_t>(r.symbol().size()), r.source_ids().data(),
                                     r.source_ids().size(), r.encoded_size(), out.data()));
  }

  void write_source(const encoder_source& s)
  {
    std::vector<std::uint8_t> out(or_packet_bound(s.size(), 0));
    emit(out, or_write_source_packet(s.id(), reinterpret_cast<const std::uint8_t*>(s.symbol().data()), s.size(),
                                     out.data()));
  }

  /// @throw overflow_error
  std::pair<ack, std::size_t> read_ack(packet&& p)
  {
    or_packet_view v;
    const std::size_t n = parse(p, v);
    ack a{source_id_list(v.ids, v.ids + v.nids), v.nb_packets};
    or_packet_view_free(&v);
    return std::make_pair(std::move(a), n);
  }

  /// @throw overflow_error
  std::pair<decoder_repair, std::size_t> read_repair(packet&& p)
  {
    or_packet_view v;
    const std::size_t n = parse(p, v);
    source_id_list ids(v.ids, v.ids + v.nids);
    or_packet_view_free(&v);
    return std::make_pair(decoder_repair{v.id, v.encoded_size, std::move(ids), std::move(p), v.symbol_size}, n);
  }

  /// @throw overflow_error
  std::pair<decoder_source, std::size_t> read_source(packet&& p)
  {
    or_packet_view v;
    const std::size_t n = parse(p, v);
    or_packet_view_free(&v);
    return std::make_pair(decoder_source{v.id, std::move(p), v.symbol_size}, n);
  }

private:
  void emit(const std::vector<std::uint8_t>& out, std::size_t n)
  {
    h_(reinterpret_cast<const char*>(out.data()), n);
    h_();
  }

  // the symbol of a source / repair is read where packet::symbol() points (7 bytes in)
  static std::size_t parse(const packet& p, or_packet_view& v)
  {
    const long n = or_parse_packet(reinterpret_cast<const std::uint8_t*>(p.data()), p.size(), &v);
    if (n == -1) throw packet_type_error{p};
    if (n < 0) throw overflow_error{};
    return static_cast<std::size_t>(n);
  }

  PacketHandler& h_;
};

}  // namespace detail
}  // namespace ntc
