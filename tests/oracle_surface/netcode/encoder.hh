// tests/oracle_surface (tests only): ntc::encoder (reference encoder.hh) = the oracle's public
// encoder (or_encoder: window, code type, rate, adaptive rate from acks, repairs, wire packets).
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>

#include "netcode/data.hh"
#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/packetizer.hh"   // the reference's header brings the detail layer along
#include "netcode/errors.hh"
#include "netcode/packet.hh"
#include "netcode/systematic.hh"

namespace ntc {

template <typename PacketHandler>
class encoder final
{
public:
  using packet_handler_type = PacketHandler;

  template <typename PacketHandler_>
  encoder(std::uint8_t galois_field_size, PacketHandler_&& h)
    : w_{galois_field_size}, h_(std::forward<PacketHandler_>(h)), e_{or_encoder_new(&emit, this)}
  {
    or_encoder_set_field(e_, galois_field_size);
  }
  ~encoder() { or_encoder_free(e_); }
  encoder(const encoder&) = delete;
  encoder& operator=(const encoder&) = delete;

  void operator()(const data& d) { operator()(data{d}); }
  void operator()(data&& d)
  {
    or_encoder_add_data(e_, reinterpret_cast<const std::uint8_t*>(d.data()), static_cast<std::uint16_t>(d.size()));
    ex_.rethrow();
  }

  std::size_t operator()(const packet& p) { return operator()(packet{p}); }
  std::size_t operator()(packet&& p)
  {
    const long n = or_encoder_add_packet(e_, reinterpret_cast<const std::uint8_t*>(p.data()), p.size());
    ex_.rethrow();
    if (n == -1) throw packet_type_error{p};
    if (n < 0) throw overflow_error{};
    return static_cast<std::size_t>(n);
  }

  void generate_repair()
  {
    or_encoder_generate_repair(e_);
    ex_.rethrow();
  }

  std::size_t window() const noexcept { return or_encoder_window(e_); }
  std::size_t nb_received_acks() const noexcept { return or_encoder_nb_received_acks(e_); }
  std::size_t nb_sent_repairs() const noexcept { return or_encoder_nb_sent_repairs(e_); }
  std::size_t nb_sent_sources() const noexcept { return or_encoder_nb_sent_sources(e_); }
  const packet_handler_type& packet_handler() const noexcept { return h_; }
  packet_handler_type& packet_handler() noexcept { return h_; }
  std::uint8_t galois_field_size() const noexcept { return w_; }

  encoder& set_code_type(systematic c) noexcept
  {
    code_ = c;
    or_encoder_set_code_type(e_, c == systematic::yes);
    return *this;
  }
  systematic code_type() const noexcept { return code_; }
  encoder& set_rate(std::size_t rate) noexcept
  {
    or_encoder_set_rate(e_, rate);
    return *this;
  }
  std::size_t rate() const noexcept { return or_encoder_rate(e_); }
  encoder& set_window_size(std::size_t sz) noexcept
  {
    window_size_ = sz;
    or_encoder_set_window_size(e_, sz);
    return *this;
  }
  std::size_t window_size() const noexcept { return window_size_; }
  encoder& set_adaptive(bool a) noexcept
  {
    adaptive_ = a;
    or_encoder_set_adaptive(e_, a);
    return *this;
  }
  bool adaptive() const noexcept { return adaptive_; }

private:
  static void emit(void* ctx, const std::uint8_t* bytes, std::size_t len)
  {
    auto* e = static_cast<encoder*>(ctx);
    try {
      e->h_(reinterpret_cast<const char*>(bytes), len);
      e->h_();
    } catch (...) {
      e->ex_.park();
    }
  }

  std::uint8_t w_;
  packet_handler_type h_;
  or_encoder* e_;
  detail::parked_exception ex_;
  systematic code_ = systematic::yes;
  std::size_t window_size_ = static_cast<std::size_t>(-1);
  bool adaptive_ = false;
};

}  // namespace ntc
