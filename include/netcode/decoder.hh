// netcode/decoder.hh -- ntc::decoder<PacketHandler, DataHandler> (reference netcode/decoder.hh).
// Header-only C++11 surface over libntc.so's decoder (netcode/c/decoder.h); reductions, peeling
// and full decodings run on the MI355X engine.  Same constructor, operators and accessors as the
// reference.
#pragma once

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <utility>

#include "netcode/detail/c_bridge.hh"
#include "netcode/detail/packetizer.hh"   // the reference's public headers expose the wire layer
#include "netcode/errors.hh"
#include "netcode/in_order.hh"
#include "netcode/packet.hh"

namespace ntc {

template <typename PacketHandler, typename DataHandler>
class decoder final
{
public:
  using packet_handler_type = PacketHandler;
  using data_handler_type = DataHandler;

  decoder(const decoder&) = delete;
  decoder& operator=(const decoder&) = delete;
  decoder(decoder&&) = delete;
  decoder& operator=(decoder&&) = delete;

  template <typename PacketHandler_, typename DataHandler_>
  decoder(std::uint8_t galois_field_size, in_order ordered, PacketHandler_&& packet_handler,
          DataHandler_&& data_handler)
    : m_galois_field_size{galois_field_size}
    , m_ack_period{std::chrono::milliseconds{100}}
    , m_ack_nb_packets{50}
    , m_packet_handler(std::forward<PacketHandler_>(packet_handler))
    , m_data_handler(std::forward<DataHandler_>(data_handler))
    , m_dec{nullptr}
  {
    ntc_packet_handler ph;
    ph.context = this;
    ph.prepare_packet = &decoder::prepare_cb;
    ph.send_packet = &decoder::send_cb;
    ntc_data_handler dh;
    dh.context = this;
    dh.read_data = &decoder::read_cb;
    m_dec = ntc_new_decoder(galois_field_size,
                            ordered == in_order::yes ? ntc_in_order_yes : ntc_in_order_no, ph, dh);
    if (!m_dec)
      throw std::runtime_error("ntc::decoder: unsupported Galois field size or no MI355X engine");
  }

  ~decoder() { ntc_delete_decoder(m_dec); }

  /// Give the decoder a source or a repair; returns the number of bytes read.
  /// @throw packet_type_error for any other packet type.
  std::size_t operator()(const packet& p) { return operator()(packet{p}); }
  std::size_t operator()(packet&& p)
  {
    ntc_error e{ntc_no_error, nullptr};
    const std::size_t n = ntc_decoder_add_packet(m_dec, m_packet.load(p.data(), p.size()), &e);
    m_pending.rethrow();
    detail::throw_on(e, &p);
    return n;
  }

  const packet_handler_type& packet_handler() const noexcept { return m_packet_handler; }
  packet_handler_type& packet_handler() noexcept { return m_packet_handler; }
  const data_handler_type& data_handler() const noexcept { return m_data_handler; }
  data_handler_type& data_handler() noexcept { return m_data_handler; }

  std::size_t nb_decoded() const noexcept { return counter(NTC_DEC_NB_DECODED); }
  std::size_t nb_failed_full_decodings() const noexcept { return counter(NTC_DEC_NB_FAILED_FULL_DECODINGS); }
  std::size_t nb_missing_sources() const noexcept { return counter(NTC_DEC_NB_MISSING_SOURCES); }
  std::size_t nb_received_repairs() const noexcept { return counter(NTC_DEC_NB_RECEIVED_REPAIRS); }
  std::size_t nb_received_sources() const noexcept { return counter(NTC_DEC_NB_RECEIVED_SOURCES); }
  std::size_t nb_sent_acks() const noexcept { return counter(NTC_DEC_NB_SENT_ACKS); }
  std::size_t nb_useless_repairs() const noexcept { return counter(NTC_DEC_NB_USELESS_REPAIRS); }

  /// Force the sending of an ack.
  void generate_ack()
  {
    ntc_error e{ntc_no_error, nullptr};
    ntc_decoder_generate_ack(m_dec, &e);
    m_pending.rethrow();
    detail::throw_on(e);
  }

  /// Send an ack if enough packets arrived or the ack period elapsed (reference decoder.hh:
  /// 231-248; also run after every delivery).
  void maybe_ack()
  {
    ntc_error e{ntc_no_error, nullptr};
    ntc_decoder_maybe_ack(m_dec, &e);
    m_pending.rethrow();
    detail::throw_on(e);
  }

  decoder& set_ack_period(std::chrono::milliseconds f) noexcept
  {
    m_ack_period = f;
    ntc_decoder_set_ack_period(m_dec, static_cast<std::size_t>(f.count()));
    return *this;
  }
  std::chrono::milliseconds ack_period() const noexcept { return m_ack_period; }

  decoder& set_ack_nb_packets(std::uint16_t nb) noexcept
  {
    m_ack_nb_packets = std::min(nb, static_cast<std::uint16_t>(128));   // decoder.hh:277
    ntc_decoder_set_ack_nb_packets(m_dec, nb);
    return *this;
  }
  std::uint16_t ack_nb_packets() const noexcept { return m_ack_nb_packets; }

  std::uint8_t galois_field_size() const noexcept { return m_galois_field_size; }

private:
  std::size_t counter(int which) const noexcept { return ntc_decoder_counter(m_dec, which); }

  static void prepare_cb(void* ctx, const char* bytes, std::size_t sz) noexcept
  {
    decoder* self = static_cast<decoder*>(ctx);
    if (self->m_pending.ex) return;
    try { self->m_packet_handler(bytes, sz); } catch (...) { self->m_pending.ex = std::current_exception(); }
  }
  static void send_cb(void* ctx) noexcept
  {
    decoder* self = static_cast<decoder*>(ctx);
    if (self->m_pending.ex) return;
    try { self->m_packet_handler(); } catch (...) { self->m_pending.ex = std::current_exception(); }
  }
  static void read_cb(void* ctx, const char* bytes, std::size_t sz) noexcept
  {
    decoder* self = static_cast<decoder*>(ctx);
    if (self->m_pending.ex) return;
    try { self->m_data_handler(bytes, sz); } catch (...) { self->m_pending.ex = std::current_exception(); }
  }

  const std::uint8_t m_galois_field_size;
  std::chrono::milliseconds m_ack_period;
  std::uint16_t m_ack_nb_packets;
  packet_handler_type m_packet_handler;
  data_handler_type m_data_handler;
  ntc_decoder_t* m_dec;
  detail::c_packet m_packet;
  detail::pending_exception m_pending;
};

}  // namespace ntc
