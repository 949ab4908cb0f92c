"""Generate netcode_amd/csrc/gf_bitslice_table.inc -- the bit-sliced GF(2^8) MAC's block table.

Bit-sliced multiply-accumulate: a lane holds 32 bytes as 8 bit-planes x_0..x_7
(plane p = bit p of every byte).  Multiplication by a constant c is GF(2)-linear on the 8 bits
of a byte, so plane p of c*x is the XOR of the input planes q whose bit p of c*alpha^q is set.
Four-Russians split: per source the 15 nonzero XOR combinations of planes 0-3 (TL) and of planes
4-7 (TH) are built once (22 XORs; singletons are the planes themselves), 30 planes Y[0..29] in
all; then output plane p of c*x is TL[a_p] ^ TH[b_p] with (a_p, b_p) the two nibbles of row p of
c's 8x8 GF(2) matrix -- one 3-input v_bitop3 per plane, <= 8 per (source, row).

The table: 256 blocks of 128 bytes, block c = the <= 8 v_bitop3 of acc ^= c*x on the
accumulator planes v[32..39], then a scalar tail that steps to the next row.  The row is chosen by
VGPR-relative addressing (s_set_gpr_idx_on SRC0|DST, M0 index 8*j: row j's planes are
v[32+8j .. 39+8j]; the table planes are src1 / src2, never relative).  The tail shifts the 8
coefficient bytes of the tile right by one byte (SCC = rows left), turns the new low byte c into
its block address (c << 7), adds 8 to the index and jumps; when no nonzero coefficient is left it
returns through s[92:93] (s_swappc at entry).  A fast copy keeps the jump target's high half
fixed; the safe copy (used only when the fast one straddles a 4 GiB boundary) propagates the
carry.  The table lives once per code object, in a never-called holder function, so every MAC
kernel shares it and its loop stays short.

Registers fixed by the table: Y[0..29] in v2..v31, accumulators v32.. (8-row tiles v32..v95,
16-row tiles v32..v159: <= 168 VGPRs, 3 waves per SIMD), s[90:91] coefficient bytes, s[92:93]
return address, s[88:89] the second half's coefficient bytes of a 16-row tile (0: none),
s[96:97] table base, s98/s99 scratch, M0 the row index.

Usage: python tools/gen_bitslice_table.py   (rewrites the .inc; commit the result)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("NTC_BS_OUT") or os.path.join(os.path.dirname(HERE), "netcode_amd", "csrc",
                                                 "gf_bitslice_table.inc")
NPLANES = 30
Y0 = 2            # first table-plane VGPR
ACC = 32          # first accumulator VGPR (row 0, plane 0)
BLOCK = 128       # bytes per block (8 x 8-byte v_bitop3 + a 7-instruction tail <= 92)
MAXROWS = 16


def gmul(a, b):
    """GF(2^8) product, polynomial 0x11D (gf-complete's default w = 8 field)."""
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def table_planes():
    """lo[v] / hi[v]: index in Y of the XOR of input planes {q in v} (q < 4) / {4 + q}; the C++
    statements that build the 22 composite planes Y[8..29] from Y[0..7]."""
    lo, hi = [None] * 16, [None] * 16
    stmts, n = [], 8
    for half, tab in ((0, lo), (4, hi)):
        for q in range(4):
            tab[1 << q] = half + q
        for v in range(3, 16):
            if v & (v - 1):
                low = v & -v
                stmts.append(f"Y[{n}] = Y[{tab[v ^ low]}] ^ Y[{tab[low]}];")
                tab[v] = n
                n += 1
    assert n == NPLANES
    return lo, hi, stmts


def block_ops(c):
    """acc ^= c * x on the (relative) accumulators v[ACC..ACC+7]: per output plane p the two
    nibbles (a_p, b_p) of row p of c's 8x8 GF(2) matrix select TL[a_p] ^ TH[b_p]."""
    lo, hi, _ = table_planes()
    cols = [gmul(c, 1 << q) for q in range(8)]
    ops = []
    for p in range(8):
        a = sum(((cols[q] >> p) & 1) << q for q in range(4))
        b = sum(((cols[4 + q] >> p) & 1) << q for q in range(4))
        acc = f"v{ACC + p}"
        if a and b:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, v{Y0 + lo[a]}, v{Y0 + hi[b]} bitop3:0x96")
        elif a or b:
            ops.append(f"v_xor_b32_e64 {acc}, {acc}, v{Y0 + (lo[a] if a else hi[b])}")
    return ops


def table(safe):
    tag = "s" if safe else "f"
    lines = [".p2align 7", f"ntc_bs_{tag}:"]
    for c in range(256):
        lab = f"ntc_bs_{tag}{c}"
        lines.append(f"{lab}:")
        tail = ["s_lshr_b64 s[90:91], s[90:91], 8", f"s_cbranch_scc0 ntc_bs_ret_{tag}",
                "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17", "s_add_u32 s98, s96, s98"]
        if safe:
            tail.append("s_addc_u32 s99, s97, 0")
        tail += ["s_add_u32 m0, m0, 8", "s_setpc_b64 s[98:99]"]
        lines += block_ops(c) + tail
        # pad to exactly BLOCK bytes: an encoding that grew is an assembler error, not a misjump
        lines.append(f".fill {BLOCK} - (. - {lab}), 1, 0")
    # end of a row run: a 16-row tile's second half (its 8 coefficient bytes in s[88:89], zero
    # for none) continues at row 8 in the same call -- one return and one call fewer per source
    lines += [f"ntc_bs_ret_{tag}:", "s_cmp_eq_u64 s[88:89], 0", f"s_cbranch_scc1 ntc_bs_out_{tag}",
              "s_mov_b64 s[90:91], s[88:89]", "s_mov_b64 s[88:89], 0", "s_set_gpr_idx_idx 64",
              "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17", "s_add_u32 s98, s96, s98"]
    if safe:
        lines.append("s_addc_u32 s99, s97, 0")
    lines += ["s_setpc_b64 s[98:99]", f"ntc_bs_out_{tag}:", "s_setpc_b64 s[92:93]"]
    return lines


def main():
    _, _, stmts = table_planes()
    o = ["// Generated by tools/gen_bitslice_table.py -- do not edit by hand.",
         "// The bit-sliced GF(2^8) MAC's shared block table and its register contract (see the",
         "// generator's docstring).",
         "#pragma once", "",
         f"constexpr int kBsY = {Y0};                  // first table-plane VGPR (Y[0])",
         f"constexpr int kBsAcc = {ACC};               // first accumulator VGPR (row 0, plane 0)",
         f"constexpr int kBsPlanes = {NPLANES};            // input planes + their XOR combinations",
         f"constexpr uint32_t kBsBlock = {BLOCK};        // bytes per block (block c at c * kBsBlock)",
         f"constexpr uint32_t kBsSpan = {256 * BLOCK};       // bytes of one table copy", "",
         "// the 22 composite planes Y[8..29] from the 8 input planes Y[0..7]",
         "#define NTC_BS_TABLES(Y) \\"]
    o += [f"  {st} \\" for st in stmts] + ["", "// the holder function's body: s_endpgm (never called), the fast table, the safe table",
                                           "#define NTC_BS_TABLE_ASM \\"]
    o.append("".join(f'  "{l}\\n" \\\n' for l in ["s_endpgm"] + table(False) + table(True)) + '  ""')
    o.append("")
    o.append("#define NTC_BS_YPINS(Y) " + ", ".join(f'[y{n}] "{{v{Y0 + n}}}"(Y[{n}])' for n in range(NPLANES)))
    for r in (8, 16):
        o.append(f"#define NTC_BS_OUTS{r}(A) " + ", ".join(
            f'[A{j}] "+{{v[{ACC + 8 * j}:{ACC + 8 * j + 7}]}}"(A[{j}])' for j in range(r)))
    open(OUT, "w").write("\n".join(o) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
