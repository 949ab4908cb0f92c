// CPU check of include/netcode/detail/packetizer.hh (reference netcode/detail/packetizer.hh).
// The reference's own packetizer test (tests/netcode/detail/test_packetizer.cc) needs Boost.Endian,
// which this image lacks, so this driver restates its cases -- round trips of acks, repairs (few,
// many, sparse, large and single source ids), sources, and the truncated-packet checks -- and adds
// the byte-exact wire KAT of SURVEY §8(c) (tests/golden/kat.json "wire_rate2_abcd_efghij").
// Exit status 0 = every check passed; a failed check prints its line and exits 1.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iterator>
#include <string>
#include <vector>

#include "netcode/detail/packetizer.hh"

using namespace ntc;

namespace {

int failures = 0;

#define CHECK(cond)                                                        \
  do {                                                                     \
    if (!(cond)) {                                                         \
      std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                          \
    }                                                                      \
  } while (0)

struct sink
{
  packet pkt;
  int ends = 0;
  void operator()(const char* p, std::size_t n) { std::copy_n(p, n, std::back_inserter(pkt)); }
  void operator()() { ++ends; }
};

std::string hex(const packet& p)
{
  static const char* d = "0123456789abcdef";
  std::string s;
  for (std::size_t i = 0; i < p.size(); ++i) {
    const auto b = static_cast<unsigned char>(p.data()[i]);
    s += d[b >> 4];
    s += d[b & 15];
  }
  return s;
}

detail::zero_byte_buffer bytes(const std::vector<unsigned char>& v)
{
  detail::zero_byte_buffer b;
  for (unsigned char c : v) b.push_back(static_cast<char>(c));
  return b;
}

void repair_round_trip(std::uint32_t id, std::uint16_t esz, detail::source_id_list ids,
                       const std::vector<unsigned char>& sym)
{
  sink h;
  detail::packetizer<sink> z{h};
  const detail::source_id_list expect = ids;
  const detail::encoder_repair in{id, esz, std::move(ids), bytes(sym)};
  z.write_repair(in);
  CHECK(h.ends == 1);
  const std::size_t total = h.pkt.size();
  const auto out = z.read_repair(std::move(h.pkt));
  CHECK(out.first.id() == id);
  CHECK(out.first.encoded_size() == esz);
  CHECK(out.first.source_ids() == expect);
  CHECK(out.first.symbol_size() == sym.size());
  CHECK(std::equal(sym.begin(), sym.end(), reinterpret_cast<const unsigned char*>(out.first.symbol())));
  // read_repair stops after the encoded size: the trailing [u16 size][symbol] copy is not parsed
  CHECK(out.second == total - 2 - sym.size());
}

packet crafted(std::uint8_t type, std::uint16_t symbol_size, std::size_t len)
{
  std::vector<char> v(len, 0);
  v[0] = static_cast<char>(type);
  v[5] = static_cast<char>(symbol_size >> 8);
  v[6] = static_cast<char>(symbol_size & 0xFF);
  return packet{v.begin(), v.end()};
}

template <typename F>
bool throws_overflow(F f)
{
  try {
    f();
  } catch (const overflow_error&) {
    return true;
  }
  return false;
}

}  // namespace

int main()
{
  {   // ack round trip
    sink h;
    detail::packetizer<sink> z{h};
    const detail::ack in{{0, 1, 2, 3}, 33};
    z.write_ack(in);
    const auto out = z.read_ack(std::move(h.pkt)).first;
    CHECK(out.source_ids() == in.source_ids());
    CHECK(out.nb_packets() == 33);
  }
  // repairs: few ids, 1024 consecutive ids (several runs of <= 255), sparse ids, ids past 2^21,
  // a single source
  repair_round_trip(42, 54, {1, 2, 3, 4}, {'a', 'b', 'c'});
  {
    detail::source_id_list many;
    for (std::uint32_t i = 0; i < 1024; ++i) many.insert(i);
    repair_round_trip(42, 3, std::move(many), {'a', 'b', 'c'});
  }
  repair_round_trip(42, 54, {0, 1, 4, 5, 6, 100, 101}, {'a', 'b', 'c'});
  {
    const std::uint32_t base = 1u << 21;
    repair_round_trip(1u << 20, 54, {base, base + 1, base + 2, base + 100, base + 101}, {'a', 'b', 'c'});
  }
  repair_round_trip(0, 33, {4242}, {'x'});
  {   // source round trip and header size (type + id + size + symbol)
    sink h;
    detail::packetizer<sink> z{h};
    const detail::encoder_source in{394839, detail::byte_buffer{'a', 'b', 'c', 'd'}};
    z.write_source(in);
    CHECK(h.pkt.size() == 1 + 4 + 2 + 4);
    const auto out = z.read_source(std::move(h.pkt)).first;
    CHECK(out.id() == 394839);
    CHECK(out.symbol_size() == 4);
    CHECK(std::equal(in.symbol().begin(), in.symbol().end(), out.symbol()));
  }
  {   // wire KAT: rate 2, data "abcd" then "efghij"
    sink h;
    detail::packetizer<sink> z{h};
    z.write_source(detail::encoder_source{0, detail::byte_buffer{'a', 'b', 'c', 'd'}});
    CHECK(hex(h.pkt) == "0200000000000461626364");
    h.pkt = packet{};
    z.write_source(detail::encoder_source{1, detail::byte_buffer{'e', 'f', 'g', 'h', 'i', 'j'}});
    CHECK(hex(h.pkt) == "0200000001000665666768696a");
    h.pkt = packet{};
    z.write_repair(detail::encoder_repair{0, 0x14, {0, 1}, bytes({0x2a, 0x23, 0x24, 0x11, 0xb9, 0xb5})});
    CHECK(hex(h.pkt) == "010000000000062a232411b9b5000200000000010001001400062a232411b9b5");
  }
  {   // truncated packets (the reference's "Prevent buffer overflow" cases)
    sink h;
    detail::packetizer<sink> z{h};
    CHECK(throws_overflow([&] { z.read_repair(crafted(1, 1024, 512)); }));
    CHECK(throws_overflow([&] { z.read_source(crafted(2, 1024, 512)); }));
    CHECK(!throws_overflow([&] { z.read_source(crafted(2, 512 - 7, 512)); }));
    CHECK(throws_overflow([&] { z.read_source(crafted(2, 512 - 7 + 1, 512)); }));
    CHECK(throws_overflow([&] { z.read_ack(packet{}); }));
  }
  if (failures) {
    std::fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  std::puts("detail_packetizer_test: all checks passed");
  return 0;
}
