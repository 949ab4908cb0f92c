// netcode/detail/packetizer.hh -- wire (de)serialisation of acks, repairs and sources (reference
// netcode/detail/packetizer.hh:34-374).  All integers big-endian.
//   ack     [u8 0][u16 nb_packets][ids]
//   repair  [u8 1][u32 id][u16 len][symbol][ids][u16 encoded size][u16 len][symbol]
//           (the symbol is written twice; readers use the first copy, which lands 16-byte
//           aligned inside the packet: packet.hh)
//   source  [u8 2][u32 id][u16 len][symbol]
//   ids     [u16 pairs + 1][u32 first]{[u8 run][u16 delta]}*: the sorted ids' successive
//           differences run-length coded (runs of <= 255 equal u32 differences, each difference
//           written on 16 bits), [u16 0] for an empty list.
// Writers stream the bytes through the packet handler h(bytes, n) and end a packet with h();
// readers take the packet (decoder_repair / decoder_source keep it: zero copy) and return the
// object with the number of bytes read, throwing overflow_error on a truncated packet.
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>

#include "netcode/detail/ack.hh"
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
  explicit packetizer(PacketHandler& h) : out_(h) {}

  void write_ack(const ack& a)
  {
    u8(static_cast<std::uint8_t>(packet_type::ack));
    u16(a.nb_packets());
    ids(a.source_ids());
    out_();
  }

  void write_repair(const encoder_repair& r)
  {
    const std::uint16_t len = static_cast<std::uint16_t>(r.symbol().size());
    u8(static_cast<std::uint8_t>(packet_type::repair));
    u32(r.id());
    u16(len);
    out_(r.symbol().data(), r.symbol().size());
    ids(r.source_ids());
    u16(r.encoded_size());
    u16(len);
    out_(r.symbol().data(), r.symbol().size());
    out_();
  }

  void write_source(const encoder_source& s)
  {
    u8(static_cast<std::uint8_t>(packet_type::source));
    u32(s.id());
    u16(static_cast<std::uint16_t>(s.symbol().size()));
    out_(s.symbol().data(), s.symbol().size());
    out_();
  }

  std::pair<ack, std::size_t> read_ack(packet&& p)
  {
    cursor c{p.data(), p.size()};
    c.u8();
    const std::uint16_t nb = c.u16();
    source_id_list list = read_ids(c);
    return {ack{std::move(list), nb}, c.consumed()};
  }

  std::pair<decoder_repair, std::size_t> read_repair(packet&& p)
  {
    cursor c{p.data(), p.size()};
    c.u8();
    const std::uint32_t id = c.u32();
    const std::uint16_t len = c.u16();
    c.skip(len);
    source_id_list list = read_ids(c);
    const std::uint16_t esz = c.u16();
    const std::size_t n = c.consumed();
    return {decoder_repair{id, esz, std::move(list), std::move(p), len}, n};
  }

  std::pair<decoder_source, std::size_t> read_source(packet&& p)
  {
    cursor c{p.data(), p.size()};
    c.u8();
    const std::uint32_t id = c.u32();
    const std::uint16_t len = c.u16();
    c.skip(len);
    const std::size_t n = c.consumed();
    return {decoder_source{id, std::move(p), len}, n};
  }

private:
  struct cursor
  {
    const char* at;
    std::size_t left;
    std::size_t used = 0;
    cursor(const char* p, std::size_t n) : at{p}, left{n} {}
    const unsigned char* take(std::size_t n)
    {
      if (left < n) throw overflow_error{};
      const unsigned char* q = reinterpret_cast<const unsigned char*>(at);
      at += n;
      left -= n;
      used += n;
      return q;
    }
    void skip(std::size_t n) { take(n); }
    std::uint8_t u8() { return *take(1); }
    std::uint16_t u16()
    {
      const unsigned char* b = take(2);
      return static_cast<std::uint16_t>((b[0] << 8) | b[1]);
    }
    std::uint32_t u32()
    {
      const unsigned char* b = take(4);
      return (std::uint32_t{b[0]} << 24) | (std::uint32_t{b[1]} << 16) | (std::uint32_t{b[2]} << 8) | b[3];
    }
    std::size_t consumed() const noexcept { return used; }
  };

  void u8(std::uint8_t x)
  {
    const char b[1] = {static_cast<char>(x)};
    out_(b, 1);
  }
  void u16(std::uint16_t x)
  {
    const char b[2] = {static_cast<char>(x >> 8), static_cast<char>(x)};
    out_(b, 2);
  }
  void u32(std::uint32_t x)
  {
    const char b[4] = {static_cast<char>(x >> 24), static_cast<char>(x >> 16), static_cast<char>(x >> 8),
                       static_cast<char>(x)};
    out_(b, 4);
  }

  void ids(const source_id_list& list)
  {
    if (list.empty()) {
      u16(0);
      return;
    }
    runs_.clear();
    for (std::size_t i = 1; i < list.size();) {          // runs of equal successive differences
      const std::uint32_t d = list[i] - list[i - 1];
      std::size_t j = i + 1;
      while (j < list.size() && list[j] - list[j - 1] == d && j - i < 255) ++j;
      runs_.emplace_back(static_cast<std::uint8_t>(j - i), d);
      i = j;
    }
    u16(static_cast<std::uint16_t>(runs_.size() + 1));
    u32(list.front());
    for (const auto& run : runs_) {
      u8(run.first);
      u16(static_cast<std::uint16_t>(run.second));
    }
  }

  source_id_list read_ids(cursor& c)
  {
    source_id_list list;
    const std::uint16_t n = c.u16();
    if (n == 0) return list;
    std::uint32_t id = c.u32();
    list.insert(id);
    for (std::uint32_t k = 1; k < n; ++k) {
      const std::uint8_t run = c.u8();
      const std::uint16_t d = c.u16();
      for (std::uint8_t t = 0; t < run; ++t) list.insert(id += d);
    }
    return list;
  }

  PacketHandler& out_;
  std::vector<std::pair<std::uint8_t, std::uint32_t>> runs_;
};

}  // namespace detail
}  // namespace ntc
