// tests/oracle_surface (tests only): code type (reference systematic.hh).
#pragma once

namespace ntc {
enum class systematic { yes, no };
}  // namespace ntc
