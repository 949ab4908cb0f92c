// netcode/detail/c_bridge.hh -- glue between the header-only C++ surface (ntc::encoder,
// ntc::decoder) and the C ABI of libntc.so (netcode/c/*.h), whose state machines restate the
// reference's and whose GF(2^8) region work runs on the MI355X engine.
#pragma once

#include <cstring>
#include <exception>
#include <new>
#include <stdexcept>
#include <string>

#include "netcode/c/data.h"
#include "netcode/c/decoder.h"
#include "netcode/c/encoder.h"
#include "netcode/c/error.h"
#include "netcode/c/ext.h"
#include "netcode/c/handlers.h"
#include "netcode/c/packet.h"
#include "netcode/errors.hh"
#include "netcode/packet.hh"

namespace ntc {
namespace detail {

// ntc_error -> the reference's exceptions (the inverse of c/detail/check_error.hh:20-67).
inline void throw_on(const ntc_error& e, const packet* p = nullptr)
{
  switch (e.type) {
    case ntc_no_error: return;
    case ntc_no_memory: throw std::bad_alloc{};
    case ntc_packet_type_error: throw packet_type_error{p ? *p : packet{}};
    case ntc_overflow_error: throw overflow_error{};
    default: throw std::runtime_error(e.message ? e.message : "netcode: unknown error");
  }
}

// One reusable C-side packet buffer (the C ABI consumes what it is given; resize revives it).
class c_packet
{
public:
  c_packet() : m_p{ntc_new_packet(0)} { if (!m_p) throw std::bad_alloc{}; }
  ~c_packet() { ntc_delete_packet(m_p); }
  c_packet(const c_packet&) = delete;
  c_packet& operator=(const c_packet&) = delete;
  ntc_packet_t* load(const char* bytes, std::size_t n)
  {
    if (n > 0xFFFF) throw overflow_error{};      // the C ABI sizes packets with uint16_t
    ntc_error e{ntc_no_error, nullptr};
    ntc_packet_resize(m_p, static_cast<uint16_t>(n), &e);
    throw_on(e);
    if (n) std::memcpy(ntc_packet_buffer(m_p), bytes, n);
    return m_p;
  }
private:
  ntc_packet_t* m_p;
};

class c_data
{
public:
  c_data() : m_d{ntc_new_data(0)} { if (!m_d) throw std::bad_alloc{}; }
  ~c_data() { ntc_delete_data(m_d); }
  c_data(const c_data&) = delete;
  c_data& operator=(const c_data&) = delete;
  ntc_data_t* load(const char* bytes, std::size_t n)
  {
    if (n > 0xFFFF) throw overflow_error{};      // symbol sizes are uint16_t (reference too)
    ntc_error e{ntc_no_error, nullptr};
    ntc_data_resize(m_d, static_cast<uint16_t>(n), &e);
    throw_on(e);
    if (n) std::memcpy(ntc_data_buffer(m_d), bytes, n);
    return m_d;
  }
private:
  ntc_data_t* m_d;
};

// Exceptions thrown by user handlers must not cross the C ABI: the trampolines park them here
// and the C++ wrapper rethrows after the C call returns.
struct pending_exception
{
  std::exception_ptr ex;
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
