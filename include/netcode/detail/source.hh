// netcode/detail/source.hh -- the source symbol types of the detail layer (reference
// netcode/detail/source.hh:11-146).
//   encoder_source  a source held by the encoder's window: id + its data (a byte_buffer).
//   decoder_source  a received or recovered source: id + the packet its symbol lives in (the
//                   symbol at packet.symbol(), 16-byte aligned, no copy out of the packet) + the
//                   symbol's size.
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
  encoder_source(std::uint32_t id, byte_buffer&& data) : id_{id}, data_{std::move(data)} {}
  encoder_source(encoder_source&&) = default;
  encoder_source& operator=(encoder_source&&) = default;
  encoder_source(const encoder_source&) = delete;
  encoder_source& operator=(const encoder_source&) = delete;

  std::uint32_t id() const noexcept { return id_; }
  const byte_buffer& symbol() const noexcept { return data_; }
  byte_buffer& symbol() noexcept { return data_; }
  std::uint16_t size() const noexcept { return static_cast<std::uint16_t>(data_.size()); }

private:
  std::uint32_t id_;
  byte_buffer data_;
};

class decoder_source final
{
public:
  decoder_source(std::uint32_t id, packet&& p, std::size_t symbol_size)
    : id_{id}, holder_{std::move(p)}, size_{static_cast<std::uint16_t>(symbol_size)}
  {}
  decoder_source(decoder_source&&) = default;
  decoder_source& operator=(decoder_source&&) = default;
  decoder_source(const decoder_source&) = delete;
  decoder_source& operator=(const decoder_source&) = delete;

  std::uint32_t id() const noexcept { return id_; }
  const char* symbol() const noexcept { return holder_.symbol(); }
  char* symbol() noexcept { return holder_.symbol(); }
  std::uint16_t symbol_size() const noexcept { return size_; }

private:
  std::uint32_t id_;
  packet holder_;
  std::uint16_t size_;
};

}  // namespace detail
}  // namespace ntc
