// Drives the header-only C++ surface (include/netcode/*.hh -> libntc.so -> MI355X engine) the way
// netcode's own programs do: an encoder/decoder pair exchanging packets through handlers, a lossy
// channel, acks, dispatch and error paths.  Prints one "ok <check>" line per passed check and a
// JSON line of counters for the lossy run (compared by tests/test_gpu_cpp_surface.py with the
// golden counters of the reference's tests/end_to_end.cc).
//
// usage: cpp_surface_test <nb_packets>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <iostream>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "netcode/decoder.hh"
#include "netcode/dispatch.hh"
#include "netcode/encoder.hh"

namespace {

#define CHECK(cond)                                                                               \
  do {                                                                                            \
    if (!(cond)) {                                                                                \
      std::cerr << "FAILED " << __LINE__ << ": " #cond "\n";                                      \
      std::exit(1);                                                                               \
    }                                                                                             \
  } while (0)

// Collects whole packets: bytes arrive through (ptr, size) calls, the packet ends with ().
struct packet_sink
{
  std::vector<std::vector<char>> done;
  std::vector<char> cur;
  void operator()(const char* p, std::size_t n) { cur.insert(cur.end(), p, p + n); }
  void operator()() { done.push_back(cur); cur.clear(); }
};

struct data_sink
{
  std::vector<std::vector<char>> got;
  void operator()(const char* p, std::size_t n) { got.emplace_back(p, p + n); }
};

// In-order checker: payload i is 1024 bytes whose u32 words all equal i.
struct ordered_check
{
  std::uint32_t expected = 0;
  std::size_t nb = 0;
  void operator()(const char* p, std::size_t n)
  {
    if (n != 1024) throw std::runtime_error("bad length");
    std::uint32_t w;
    for (std::size_t o = 0; o < n; o += 4) {
      std::memcpy(&w, p + o, 4);
      if (w != expected) throw std::runtime_error("out of order or corrupted");
    }
    ++expected;
    ++nb;
  }
};

struct throwing_sink
{
  void operator()(const char*, std::size_t) { throw std::logic_error("handler says no"); }
  void operator()() {}
};

// Good/bad two-state channel with libstdc++'s default engine and a 1..100 draw (the loss model
// the reference's end_to_end uses, tools/loss/burst.hh semantics).
class gilbert
{
public:
  gilbert(unsigned good, unsigned bad) : m_good{good}, m_bad{bad} {}
  bool lost()
  {
    const unsigned x = m_dist(m_gen);
    if (!m_in_bad) {
      if (x < m_good) return false;
      m_in_bad = true;
      return true;
    }
    if (x < m_bad) return true;
    m_in_bad = false;
    return false;
  }
private:
  std::default_random_engine m_gen;
  std::uniform_int_distribution<unsigned> m_dist{1, 100};
  unsigned m_good, m_bad;
  bool m_in_bad = false;
};

void basic()
{
  ntc::encoder<packet_sink> enc{8, packet_sink{}};
  enc.set_window_size(32);
  ntc::decoder<packet_sink, data_sink> dec{8, ntc::in_order::yes, packet_sink{}, data_sink{}};
  dec.set_ack_period(std::chrono::milliseconds{200});
  enc(ntc::data{'a', 'b', 'c'});
  const auto& pk = enc.packet_handler().done;
  CHECK(pk.size() == 1);
  dec(ntc::packet{pk[0].begin(), pk[0].end()});
  CHECK(dec.data_handler().got.size() == 1);
  CHECK(std::string(dec.data_handler().got[0].begin(), dec.data_handler().got[0].end()) == "abc");
  CHECK(enc.window() == 1 && enc.nb_sent_sources() == 1 && dec.nb_received_sources() == 1);
  std::cout << "ok basic\n";
}

void repair_recovers_lost_source()
{
  ntc::encoder<packet_sink> enc{8, packet_sink{}};
  enc.set_rate(2);
  ntc::decoder<packet_sink, data_sink> dec{8, ntc::in_order::no, packet_sink{}, data_sink{}};
  enc(ntc::data{'a', 'b', 'c', 'd'});
  enc(ntc::data{'e', 'f', 'g', 'h', 'i', 'j'});
  const auto& pk = enc.packet_handler().done;
  CHECK(pk.size() == 3);                           // 2 sources + 1 repair (rate 2)
  CHECK(pk[2][0] == 1 && pk[0][0] == 2);           // repair / source type bytes
  dec(ntc::packet{pk[1].begin(), pk[1].end()});    // first source lost
  dec(ntc::packet{pk[2].begin(), pk[2].end()});
  CHECK(dec.nb_decoded() == 1 && dec.data_handler().got.size() == 2);
  CHECK(std::string(dec.data_handler().got[1].begin(), dec.data_handler().got[1].end()) == "abcd");
  std::cout << "ok repair_recovers_lost_source\n";
}

void dispatch_and_errors()
{
  ntc::encoder<packet_sink> enc{8, packet_sink{}};
  ntc::decoder<packet_sink, data_sink> dec{8, ntc::in_order::yes, packet_sink{}, data_sink{}};
  enc(ntc::data{'x', 'y'});
  auto src = enc.packet_handler().done.back();
  ntc::dispatch(enc, dec, ntc::packet{src.begin(), src.end()});
  CHECK(dec.nb_received_sources() == 1);
  dec.generate_ack();
  auto ack = dec.packet_handler().done.back();
  CHECK(ack[0] == 0);
  ntc::dispatch(enc, dec, ntc::packet{ack.begin(), ack.end()});
  CHECK(enc.nb_received_acks() == 1 && enc.window() == 0);
  bool thrown = false;
  try { dec(ntc::packet{ack.begin(), ack.end()}); } catch (const ntc::packet_type_error& e) {
    thrown = e.error_packet.size() == ack.size();
  }
  CHECK(thrown);
  thrown = false;
  try { enc(ntc::packet{src.begin(), src.end()}); } catch (const ntc::packet_type_error&) { thrown = true; }
  CHECK(thrown);
  thrown = false;
  try { ntc::dispatch(enc, dec, ntc::packet{char(7), char(0)}); } catch (const ntc::packet_type_error&) { thrown = true; }
  CHECK(thrown);
  // an exception thrown by a user handler reaches the caller unchanged
  ntc::encoder<throwing_sink> bad{8, throwing_sink{}};
  thrown = false;
  try { bad(ntc::data{'z'}); } catch (const std::logic_error& e) { thrown = std::string(e.what()) == "handler says no"; }
  CHECK(thrown);
  // setters / getters
  enc.set_rate(3).set_window_size(9).set_adaptive(false).set_code_type(ntc::systematic::no);
  CHECK(enc.rate() == 3 && enc.window_size() == 9 && !enc.adaptive() && enc.code_type() == ntc::systematic::no);
  dec.set_ack_nb_packets(500);
  CHECK(dec.ack_nb_packets() == 128);
  CHECK(enc.galois_field_size() == 8);
  {  // every field size netcode supports (galois_field.hh:39); anything else is rejected
    ntc::encoder<packet_sink> e16{16, packet_sink{}};
    CHECK(e16.galois_field_size() == 16);
    ntc::encoder<packet_sink> e32{32, packet_sink{}};
    CHECK(e32.galois_field_size() == 32);
    bool unsupported = false;
    try { ntc::encoder<packet_sink> e7{7, packet_sink{}}; } catch (const std::runtime_error&) { unsupported = true; }
    CHECK(unsupported);
  }
  std::cout << "ok dispatch_and_errors\n";
}

void packet_api()
{
  ntc::packet p{'a', 'b', 'c'};
  CHECK(p.size() == 3 && p[1] == 'b' && !p.empty());
  p.push_back('d');
  p.resize(6, 'z');
  CHECK(p.size() == 6 && p[5] == 'z');
  ntc::packet q(4, 'q');
  q.assign({'1', '2'});
  CHECK(q.size() == 2 && q == ntc::packet({'1', '2'}));
  ntc::data d(16);
  CHECK(reinterpret_cast<std::uintptr_t>(d.data()) % 16 == 0);
  std::cout << "ok packet_api\n";
}

// The reference's tests/end_to_end.cc loop restated: 1024-B payloads, rate 5 (default), in-order
// decoder, an ack whenever received sources + repairs is a multiple of 50, one loss model shared
// by both directions.
void lossy_stream(std::uint32_t nb_packets)
{
  ntc::encoder<packet_sink> enc{8, packet_sink{}};
  ntc::decoder<packet_sink, ordered_check> dec{8, ntc::in_order::yes, packet_sink{}, ordered_check{}};
  dec.set_ack_period(std::chrono::milliseconds{0});
  gilbert loss{95, 5};
  std::size_t lost_to_dec = 0, lost_to_enc = 0;
  for (std::uint32_t id = 0; id < nb_packets; ++id) {
    ntc::data d(1024);
    for (std::size_t o = 0; o < 1024; o += 4) std::memcpy(d.data() + o, &id, 4);
    enc(std::move(d));
    for (const auto& pkt : enc.packet_handler().done) {
      if (!loss.lost()) dec(ntc::packet{pkt.begin(), pkt.end()});
      else ++lost_to_dec;
    }
    enc.packet_handler().done.clear();
    if ((dec.nb_received_sources() + dec.nb_received_repairs()) % 50 == 0) {
      dec.generate_ack();
      for (const auto& pkt : dec.packet_handler().done) {
        if (!loss.lost()) enc(ntc::packet{pkt.begin(), pkt.end()});
        else ++lost_to_enc;
      }
    }
    dec.packet_handler().done.clear();
  }
  std::cout << "{\"sent\": " << nb_packets << ", \"lost\": " << lost_to_dec
            << ", \"received_repairs\": " << dec.nb_received_repairs()
            << ", \"received_sources\": " << dec.nb_received_sources()
            << ", \"useless_repairs\": " << dec.nb_useless_repairs()
            << ", \"decoded\": " << dec.nb_decoded()
            << ", \"handled\": " << dec.data_handler().nb << "}\n";
}

}  // namespace

int main(int argc, char** argv)
{
  const std::uint32_t n = argc > 1 ? static_cast<std::uint32_t>(std::atoi(argv[1])) : 1000u;
  packet_api();
  basic();
  repair_recovers_lost_source();
  dispatch_and_errors();
  lossy_stream(n);
  return 0;
}
