// netcode/encoder.hh -- ntc::encoder<PacketHandler> (reference netcode/encoder.hh:28-399).
// Header-only C++11 surface over libntc.so's encoder (netcode/c/encoder.h); repairs are built
// by the MI355X engine.  Same constructor, operators, getters and setters as the reference.
#pragma once

#include <cstddef>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <utility>

#include "netcode/data.hh"
#include "netcode/detail/c_bridge.hh"
#include "netcode/detail/packetizer.hh"   // the reference's public headers expose the wire layer
#include "netcode/errors.hh"
#include "netcode/packet.hh"
#include "netcode/systematic.hh"

namespace ntc {

template <typename PacketHandler>
class encoder final
{
public:
  using packet_handler_type = PacketHandler;

  encoder(const encoder&) = delete;
  encoder& operator=(const encoder&) = delete;
  encoder(encoder&&) = delete;
  encoder& operator=(encoder&&) = delete;

  /// galois_field_size: 4, 8, 16 or 32 (galois_field.hh:39).
  template <typename PacketHandler_>
  encoder(std::uint8_t galois_field_size, PacketHandler_&& packet_handler)
    : m_galois_field_size{galois_field_size}
    , m_code_type{systematic::yes}
    , m_window_size{std::numeric_limits<std::size_t>::max()}
    , m_adaptive{false}
    , m_packet_handler(std::forward<PacketHandler_>(packet_handler))
    , m_enc{nullptr}
  {
    ntc_packet_handler h;
    h.context = this;
    h.prepare_packet = &encoder::prepare_cb;
    h.send_packet = &encoder::send_cb;
    m_enc = ntc_new_encoder(galois_field_size, h);
    if (!m_enc)
      throw std::runtime_error("ntc::encoder: unsupported Galois field size or no MI355X engine");
  }

  ~encoder() { ntc_delete_encoder(m_enc); }

  /// Give the encoder a new data (sent as a source if systematic; may trigger a repair).
  void operator()(const data& d) { operator()(data{d}); }
  void operator()(data&& d)
  {
    ntc_error e{ntc_no_error, nullptr};
    ntc_encoder_add_data(m_enc, m_data.load(d.data(), d.size()), &e);
    m_pending.rethrow();
    detail::throw_on(e);
  }

  /// Notify the encoder of an incoming ack; returns the number of bytes read.
  std::size_t operator()(const packet& p) { return operator()(packet{p}); }
  std::size_t operator()(packet&& p)
  {
    ntc_error e{ntc_no_error, nullptr};
    const std::size_t n = ntc_encoder_add_packet(m_enc, m_packet.load(p.data(), p.size()), &e);
    m_pending.rethrow();
    detail::throw_on(e, &p);
    return n;
  }

  std::size_t window() const noexcept { return ntc_encoder_window(m_enc); }
  std::size_t nb_received_acks() const noexcept { return ntc_encoder_counter(m_enc, NTC_ENC_NB_RECEIVED_ACKS); }
  std::size_t nb_sent_repairs() const noexcept { return ntc_encoder_counter(m_enc, NTC_ENC_NB_SENT_REPAIRS); }
  std::size_t nb_sent_sources() const noexcept { return ntc_encoder_counter(m_enc, NTC_ENC_NB_SENT_SOURCES); }

  const packet_handler_type& packet_handler() const noexcept { return m_packet_handler; }
  packet_handler_type& packet_handler() noexcept { return m_packet_handler; }

  /// Force the sending of a repair (no-op on an empty window).
  void generate_repair()
  {
    ntc_error e{ntc_no_error, nullptr};
    ntc_encoder_generate_repair(m_enc, &e);
    m_pending.rethrow();
    detail::throw_on(e);
  }

  std::uint8_t galois_field_size() const noexcept { return m_galois_field_size; }

  encoder& set_code_type(systematic c) noexcept
  {
    m_code_type = c;
    ntc_encoder_set_code_type(m_enc, c == systematic::yes ? ntc_systematic_yes : ntc_systematic_no);
    return *this;
  }
  systematic code_type() const noexcept { return m_code_type; }

  encoder& set_rate(std::size_t rate) noexcept
  {
    ntc_encoder_set_rate(m_enc, rate);
    return *this;
  }
  /// The current rate (changes by itself when adaptive).
  std::size_t rate() const noexcept { return ntc_encoder_counter(m_enc, NTC_ENC_RATE); }

  encoder& set_window_size(std::size_t sz) noexcept
  {
    m_window_size = sz;
    ntc_encoder_set_window_size(m_enc, sz);
    return *this;
  }
  std::size_t window_size() const noexcept { return m_window_size; }

  encoder& set_adaptive(bool adaptive) noexcept
  {
    m_adaptive = adaptive;
    ntc_encoder_set_adaptive(m_enc, adaptive);
    return *this;
  }
  bool adaptive() const noexcept { return m_adaptive; }

private:
  static void prepare_cb(void* ctx, const char* bytes, std::size_t sz) noexcept
  {
    encoder* self = static_cast<encoder*>(ctx);
    if (self->m_pending.ex) return;
    try { self->m_packet_handler(bytes, sz); } catch (...) { self->m_pending.ex = std::current_exception(); }
  }
  static void send_cb(void* ctx) noexcept
  {
    encoder* self = static_cast<encoder*>(ctx);
    if (self->m_pending.ex) return;
    try { self->m_packet_handler(); } catch (...) { self->m_pending.ex = std::current_exception(); }
  }

  const std::uint8_t m_galois_field_size;
  systematic m_code_type;
  std::size_t m_window_size;
  bool m_adaptive;
  packet_handler_type m_packet_handler;
  ntc_encoder_t* m_enc;
  detail::c_data m_data;
  detail::c_packet m_packet;
  detail::pending_exception m_pending;
};

}  // namespace ntc
