// tests/oracle_surface -- TEST INFRASTRUCTURE ONLY.  The reference's C++ API (public ntc::encoder /
// ntc::decoder and the ntc::detail layer) as thin bindings over the CPU oracle
// (oracle/ntc_oracle.c), so that the reference's OWN test programs -- its Catch suites and
// tests/end_to_end.cc, compiled unmodified -- check the checker itself.  Containers are plain
// std:: types; every semantic step (field arithmetic, coefficients, repair building, the decoder
// state machine, inversion, the wire format, acks, rates) is the oracle's C code.  Nothing under
// netcode_amd/ or include/ includes this tree, and this tree includes nothing from them.
#pragma once

#include <exception>

#include "ntc_oracle.h"

namespace ntc {
namespace detail {

// Exceptions thrown by user handlers must not unwind through the oracle's C frames: the
// trampolines park them and the C++ wrapper rethrows once the C call has returned.
struct parked_exception
{
  std::exception_ptr ex;
  void park() noexcept { if (!ex) ex = std::current_exception(); }
  void rethrow()
  {
    if (ex) {
      std::exception_ptr e = ex;
      ex = nullptr;
      std::rethrow_exception(e);
    }
  }
};

}  // namespace detail
}  // namespace ntc
