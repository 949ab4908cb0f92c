// netcode/errors.hh -- exceptions of the C++ surface (reference netcode/errors.hh).
#pragma once

#include <exception>
#include <stdexcept>
#include <string>
#include <utility>

#include "netcode/packet.hh"

namespace ntc {

/// Thrown when a packet's type could not be handled (e.g. an ack given to a decoder).
struct packet_type_error : public std::exception
{
  packet_type_error(packet p) : error_packet{std::move(p)} {}
  const char* what() const noexcept override { return "ntc::packet_type_error"; }
  packet error_packet;
};

/// Thrown when a malformed packet would have been read past its end.
struct overflow_error : public std::exception
{
  const char* what() const noexcept override { return "ntc::overflow_error"; }
};

}  // namespace ntc
