// tests/oracle_surface (tests only): ntc::decoder (reference decoder.hh) = the oracle's public
// decoder (or_decoder: counters, in-order delivery, acks by packet count and period).
#pragma once

#include <chrono>
#include <cstddef>
#include <cstdint>
#include <utility>

#include "netcode/detail/oracle_bind.hh"
#include "netcode/detail/packetizer.hh"   // the reference's header brings the detail layer along
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

  template <typename PacketHandler_, typename DataHandler_>
  decoder(std::uint8_t galois_field_size, in_order ordered, PacketHandler_&& ph, DataHandler_&& dh)
    : ph_(std::forward<PacketHandler_>(ph)), dh_(std::forward<DataHandler_>(dh)),
      d_{or_decoder_new(ordered == in_order::yes, &emit, this, &deliver, this)}
  {
    or_decoder_set_field(d_, galois_field_size);
  }
  ~decoder() { or_decoder_free(d_); }
  decoder(const decoder&) = delete;
  decoder& operator=(const decoder&) = delete;

  std::size_t operator()(const packet& p) { return operator()(packet{p}); }
  std::size_t operator()(packet&& p)
  {
    const long n = or_decoder_add_packet(d_, reinterpret_cast<const std::uint8_t*>(p.data()), p.size());
    ex_.rethrow();
    if (n == -1) throw packet_type_error{p};
    if (n < 0) throw overflow_error{};
    return static_cast<std::size_t>(n);
  }

  const packet_handler_type& packet_handler() const noexcept { return ph_; }
  packet_handler_type& packet_handler() noexcept { return ph_; }
  const data_handler_type& data_handler() const noexcept { return dh_; }
  data_handler_type& data_handler() noexcept { return dh_; }

  std::size_t nb_decoded() const noexcept { return or_decoder_counter(d_, 0); }
  std::size_t nb_failed_full_decodings() const noexcept { return or_decoder_counter(d_, 1); }
  std::size_t nb_missing_sources() const noexcept { return or_decoder_counter(d_, 2); }
  std::size_t nb_received_repairs() const noexcept { return or_decoder_counter(d_, 3); }
  std::size_t nb_received_sources() const noexcept { return or_decoder_counter(d_, 4); }
  std::size_t nb_sent_acks() const noexcept { return or_decoder_counter(d_, 5); }
  std::size_t nb_useless_repairs() const noexcept { return or_decoder_counter(d_, 6); }

  void generate_ack()
  {
    or_decoder_generate_ack(d_);
    ex_.rethrow();
  }
  void maybe_ack()
  {
    or_decoder_maybe_ack(d_);
    ex_.rethrow();
  }

  decoder& set_ack_period(std::chrono::milliseconds f) noexcept
  {
    period_ = f;
    or_decoder_set_ack_period_ms(d_, static_cast<long>(f.count()));
    return *this;
  }
  std::chrono::milliseconds ack_period() const noexcept { return period_; }
  decoder& set_ack_nb_packets(std::uint16_t nb) noexcept
  {
    nb_ = nb < 128 ? nb : 128;
    or_decoder_set_ack_nb_packets(d_, nb);
    return *this;
  }
  std::uint16_t ack_nb_packets() const noexcept { return nb_; }

private:
  static void emit(void* ctx, const std::uint8_t* bytes, std::size_t len)
  {
    auto* d = static_cast<decoder*>(ctx);
    try {
      d->ph_(reinterpret_cast<const char*>(bytes), len);
      d->ph_();
    } catch (...) {
      d->ex_.park();
    }
  }
  static void deliver(void* ctx, std::uint32_t, const std::uint8_t* bytes, std::size_t len)
  {
    auto* d = static_cast<decoder*>(ctx);
    try {
      d->dh_(reinterpret_cast<const char*>(bytes), len);
    } catch (...) {
      d->ex_.park();
    }
  }

  packet_handler_type ph_;
  data_handler_type dh_;
  or_decoder* d_;
  detail::parked_exception ex_;
  std::chrono::milliseconds period_{100};
  std::uint16_t nb_ = 50;
};

}  // namespace ntc
