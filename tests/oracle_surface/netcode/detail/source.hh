// tests/oracle_surface (tests only): encoder_source / decoder_source (reference detail/source.hh).
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>

#include "netcode/detail/buffer.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

class encoder_source final
{
public:
  encoder_source(const encoder_source&) = delete;
  encoder_source& operator=(const encoder_source&) = delete;
  encoder_source(encoder_source&&) = default;
  encoder_source& operator=(encoder_source&&) = default;

  encoder_source(std::uint32_t id, byte_buffer&& symbol) : id_{id}, sym_{std::move(symbol)} {}

  std::uint32_t id() const noexcept { return id_; }
  const byte_buffer& symbol() const noexcept { return sym_; }
  byte_buffer& symbol() noexcept { return sym_; }
  std::uint16_t size() const noexcept { return static_cast<std::uint16_t>(sym_.size()); }

private:
  std::uint32_t id_;
  byte_buffer sym_;
};

class decoder_source final
{
public:
  decoder_source(const decoder_source&) = delete;
  decoder_source& operator=(const decoder_source&) = delete;
  decoder_source(decoder_source&&) = default;
  decoder_source& operator=(decoder_source&&) = default;

  // the symbol is p.symbol(): a received packet's payload, or a bare symbol packet
  decoder_source(std::uint32_t id, packet&& p, std::size_t symbol_size)
    : id_{id}, p_{std::move(p)}, size_{static_cast<std::uint16_t>(symbol_size)}
  {}

  std::uint32_t id() const noexcept { return id_; }
  const char* symbol() const noexcept { return p_.symbol(); }
  char* symbol() noexcept { return p_.symbol(); }
  std::uint16_t symbol_size() const noexcept { return size_; }

private:
  std::uint32_t id_;
  packet p_;
  std::uint16_t size_;
};

}  // namespace detail
}  // namespace ntc
