// netcode/in_order.hh -- reference netcode/in_order.hh.
#pragma once

namespace ntc {

/// Whether a decoder delivers data in source-id order.
enum class in_order { yes, no };

}  // namespace ntc
