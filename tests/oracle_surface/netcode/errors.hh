// tests/oracle_surface (tests only): the reference's exceptions (errors.hh).
#pragma once

#include <exception>
#include <utility>

#include "netcode/packet.hh"

namespace ntc {

struct packet_type_error : public std::exception
{
  packet_type_error(packet p) : error_packet{std::move(p)} {}
  packet error_packet;
};

struct overflow_error : public std::exception
{};

}  // namespace ntc
