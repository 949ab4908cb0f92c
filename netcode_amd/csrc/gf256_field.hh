// gf256_field.hh -- compile-time GF(2^8) tables (polynomial 0x11D) for the MI355X engine.
//
// The reference gets its field from gf-complete's gf_init_easy(&gf, 8)
// (netcode/detail/galois_field.hh:35-44); gf-complete's w = 8 default polynomial is 0x11D.
// Everything the device needs is generated here by constexpr evaluation, so the tables are part
// of the code object (no host upload, no runtime initialisation race).
#pragma once

#include <cstdint>

namespace ntcgpu {

struct FieldTables {
  uint8_t exp[512];
  uint8_t log[256];
};

constexpr FieldTables make_field_tables()
{
  FieldTables t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(x);
    t.exp[i + 255] = static_cast<uint8_t>(x);
    t.log[x] = static_cast<uint8_t>(i);
    x <<= 1;
    if (x & 0x100u) x ^= 0x11Du;
  }
  t.exp[510] = t.exp[0];
  t.exp[511] = t.exp[1];
  t.log[0] = 0;
  return t;
}

constexpr FieldTables kField = make_field_tables();

constexpr uint8_t field_mul(uint8_t a, uint8_t b)
{
  return (a == 0 || b == 0) ? 0 : kField.exp[kField.log[a] + kField.log[b]];
}

constexpr uint8_t field_inv(uint8_t a) { return kField.exp[(255 - kField.log[a]) % 255]; }

// Per-coefficient v_perm_b32 lookup tables.  A byte x is split 3/3/2 bits:
//   c*x = c*(x & 7) ^ c*(x & 0x38) ^ c*(x & 0xC0)
// and each part is an 8-entry (or 4-entry) byte table selected by one v_perm_b32 for four bytes
// at once.  Word layout per coefficient c (8 dwords, 32-B aligned):
//   w[0] = {c*0, c*1, c*2, c*3}         w[1] = {c*4 .. c*7}        (bits 0-2)
//   w[2] = {c*0, c*8, c*16, c*24}       w[3] = {c*32 .. c*56}      (bits 3-5)
//   w[4] = {c*0, c*64, c*128, c*192}                               (bits 6-7)
struct PermTables {
  uint32_t w[256][8];
};

constexpr uint32_t pack4(uint8_t a, uint8_t b, uint8_t c, uint8_t d)
{
  return uint32_t(a) | (uint32_t(b) << 8) | (uint32_t(c) << 16) | (uint32_t(d) << 24);
}

constexpr PermTables make_perm_tables()
{
  PermTables t{};
  for (int c = 0; c < 256; ++c) {
    const uint8_t cc = static_cast<uint8_t>(c);
    t.w[c][0] = pack4(field_mul(cc, 0), field_mul(cc, 1), field_mul(cc, 2), field_mul(cc, 3));
    t.w[c][1] = pack4(field_mul(cc, 4), field_mul(cc, 5), field_mul(cc, 6), field_mul(cc, 7));
    t.w[c][2] = pack4(field_mul(cc, 0), field_mul(cc, 8), field_mul(cc, 16), field_mul(cc, 24));
    t.w[c][3] = pack4(field_mul(cc, 32), field_mul(cc, 40), field_mul(cc, 48), field_mul(cc, 56));
    t.w[c][4] = pack4(field_mul(cc, 0), field_mul(cc, 64), field_mul(cc, 128), field_mul(cc, 192));
  }
  return t;
}

// The same tables for the inverse of every coefficient (entry 0 stays all-zero): dividing by a
// pivot is one lookup away.
constexpr PermTables make_inv_perm_tables()
{
  PermTables t{};
  const PermTables p = make_perm_tables();
  for (int c = 1; c < 256; ++c)
    for (int e = 0; e < 8; ++e) t.w[c][e] = p.w[field_inv(static_cast<uint8_t>(c))][e];
  return t;
}

// netcode/detail/galois_field.hh:143-158 (w = 8): uint32 wraparound, then % 255 + 1.
__host__ __device__ constexpr inline uint32_t coefficient(uint32_t repair_id, uint32_t src_id)
{
  return (((repair_id + 1u) + (src_id + 1u)) * (repair_id + 1u)) % 255u + 1u;
}

}  // namespace ntcgpu
