// tests/oracle_surface (tests only): in-order delivery switch (reference in_order.hh).
#pragma once

namespace ntc {
enum class in_order { yes, no };
}  // namespace ntc
