// tests/oracle_surface (tests only): encoder_repair / decoder_repair (reference detail/repair.hh).
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
  encoder_repair(const encoder_repair&) = delete;
  encoder_repair& operator=(const encoder_repair&) = delete;
  encoder_repair(encoder_repair&&) = default;
  encoder_repair& operator=(encoder_repair&&) = default;

  explicit encoder_repair(std::uint32_t id) : id_{id}, esz_{0} {}
  encoder_repair(std::uint32_t id, std::uint16_t encoded_size, source_id_list&& ids, zero_byte_buffer&& sym)
    : id_{id}, ids_{std::move(ids)}, esz_{encoded_size}, sym_{std::move(sym)}
  {}

  std::uint32_t id() const noexcept { return id_; }
  std::uint32_t& id() noexcept { return id_; }
  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  const zero_byte_buffer& symbol() const noexcept { return sym_; }
  zero_byte_buffer& symbol() noexcept { return sym_; }
  std::uint16_t encoded_size() const noexcept { return esz_; }
  std::uint16_t& encoded_size() noexcept { return esz_; }
  void reset() noexcept
  {
    ids_.clear();
    sym_.clear();
  }

private:
  std::uint32_t id_;
  source_id_list ids_;
  std::uint16_t esz_;
  zero_byte_buffer sym_;
};

class decoder_repair final
{
public:
  decoder_repair(const decoder_repair&) = delete;
  decoder_repair& operator=(const decoder_repair&) = delete;
  decoder_repair(decoder_repair&&) = default;
  decoder_repair& operator=(decoder_repair&&) = default;

  decoder_repair(std::uint32_t id, std::uint16_t encoded_size, source_id_list&& ids, packet&& p,
                 std::size_t symbol_size)
    : id_{id}, ids_{std::move(ids)}, esz_{encoded_size}, p_{std::move(p)},
      size_{static_cast<std::uint16_t>(symbol_size)}
  {}

  std::uint32_t id() const noexcept { return id_; }
  std::uint32_t& id() noexcept { return id_; }
  const source_id_list& source_ids() const noexcept { return ids_; }
  source_id_list& source_ids() noexcept { return ids_; }
  const char* symbol() const noexcept { return p_.symbol(); }
  char* symbol() noexcept { return p_.symbol(); }
  std::uint16_t encoded_size() const noexcept { return esz_; }
  std::uint16_t& encoded_size() noexcept { return esz_; }
  std::uint16_t symbol_size() const noexcept { return size_; }

private:
  std::uint32_t id_;
  source_id_list ids_;
  std::uint16_t esz_;
  packet p_;
  std::uint16_t size_;
};

}  // namespace detail
}  // namespace ntc
