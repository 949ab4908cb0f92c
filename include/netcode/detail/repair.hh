// netcode/detail/repair.hh -- the repair symbol types of the detail layer (reference
// netcode/detail/repair.hh:13-258).
//   encoder_repair  a repair being built: id, the ids of the sources it combines, the encoded
//                   (coded) size and a zero-initialised symbol buffer, reused between repairs.
//   decoder_repair  a received repair: id, the ids of the sources it still combines (shrinks as
//                   known sources are removed), the encoded size (reduced alongside), and the
//                   packet holding its symbol -- reduced in place at packet.symbol(), like the
//                   reference (detail/decoder.cc:393-408).
#pragma once

#include <cstddef>
#include <cstdint>
#include <utility>

#include "netcode/detail/buffer.hh"
#include "netcode/detail/source_id_list.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

class encoder_repair final
{
public:
  explicit encoder_repair(std::uint32_t id) : id_{id}, encoded_size_{0} {}
  /// Test constructor (reference repair.hh:39-45).
  encoder_repair(std::uint32_t id, std::uint16_t encoded_size, source_id_list&& ids,
                 zero_byte_buffer&& symbol)
    : id_{id}, ids_{std::move(ids)}, encoded_size_{encoded_size}, symbol_{std::move(symbol)}
  {}
  encoder_repair(encoder_repair&&) = default;
  encoder_repair& operator=(encoder_repair&&) = default;
  encoder_repair(const encoder_repair&) = delete;
  encoder_repair& operator=(const encoder_repair&) = delete;

  std::uint32_t id() const noexcept { return id_; }
  std::uint32_t& id() noexcept { return id_; }
  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  std::uint16_t encoded_size() const noexcept { return encoded_size_; }
  std::uint16_t& encoded_size() noexcept { return encoded_size_; }
  const zero_byte_buffer& symbol() const noexcept { return symbol_; }
  zero_byte_buffer& symbol() noexcept { return symbol_; }

  /// Forget the sources and the symbol (the id and encoded size are rewritten by the encoder).
  void reset() noexcept
  {
    ids_.clear();
    symbol_.clear();
  }

private:
  std::uint32_t id_;
  source_id_list ids_;
  std::uint16_t encoded_size_;
  zero_byte_buffer symbol_;
};

class decoder_repair final
{
public:
  decoder_repair(std::uint32_t id, std::uint16_t encoded_size, source_id_list&& ids, packet&& p,
                 std::size_t symbol_size)
    : id_{id}, ids_{std::move(ids)}, encoded_size_{encoded_size}, holder_{std::move(p)},
      size_{static_cast<std::uint16_t>(symbol_size)}
  {}
  decoder_repair(decoder_repair&&) = default;
  decoder_repair& operator=(decoder_repair&&) = default;
  decoder_repair(const decoder_repair&) = delete;
  decoder_repair& operator=(const decoder_repair&) = delete;

  std::uint32_t id() const noexcept { return id_; }
  std::uint32_t& id() noexcept { return id_; }
  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  std::uint16_t encoded_size() const noexcept { return encoded_size_; }
  std::uint16_t& encoded_size() noexcept { return encoded_size_; }
  const char* symbol() const noexcept { return holder_.symbol(); }
  char* symbol() noexcept { return holder_.symbol(); }
  std::uint16_t symbol_size() const noexcept { return size_; }

private:
  std::uint32_t id_;
  source_id_list ids_;
  std::uint16_t encoded_size_;
  packet holder_;
  std::uint16_t size_;
};

}  // namespace detail
}  // namespace ntc
