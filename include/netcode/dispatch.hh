// netcode/dispatch.hh -- route an incoming packet to an encoder (acks) or a decoder (sources,
// repairs) by its type byte (reference netcode/dispatch.hh; packet types of
// detail/packet_type.hh: 0 ack, 1 repair, 2 source).
#pragma once

#include <cstddef>
#include <utility>

#include "netcode/decoder.hh"
#include "netcode/encoder.hh"
#include "netcode/errors.hh"
#include "netcode/packet.hh"

namespace ntc {

/// @throw packet_type_error if the type could not have been read.
template <typename Encoder, typename Decoder>
std::size_t dispatch(Encoder& encoder, Decoder& decoder, packet&& p)
{
  if (p.empty()) throw packet_type_error{std::move(p)};
  switch (static_cast<unsigned char>(p[0])) {
    case 0: return encoder(std::move(p));
    case 1:
    case 2: return decoder(std::move(p));
    default: throw packet_type_error{std::move(p)};
  }
}

}  // namespace ntc
