// netcode/systematic.hh -- reference netcode/systematic.hh.
#pragma once

namespace ntc {

/// Whether a code sends sources in clear (systematic) or only repairs.
enum class systematic { yes, no };

}  // namespace ntc
