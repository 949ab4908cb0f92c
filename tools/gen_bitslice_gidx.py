"""Generate netcode_amd/csrc/gf_bitslice_gidx.inc -- the shared-table bit-sliced MAC chain.

Same arithmetic as tools/gen_bitslice_chain.py (a lane's 32 bytes as 8 bit-planes, the Four-
Russians tables TL / TH of planes 0-3 / 4-7 in Y[8..29]; plane p of c*x = TL[a_p] ^ TH[b_p]),
but one dispatch per (source, row) instead of two, and ONE table of 256 blocks for all rows:

* block c (c = 0..255) is the full-byte multiply-accumulate acc ^= c*x -- at most 8 v_bitop3 on
  the accumulator planes v[64..71] -- written once;
* the row is selected by VGPR-relative addressing (s_set_gpr_idx_on, SRC0 + DST relative): with
  index 8j the block's v64..v71 become row j's accumulators v[64+8j .. 71+8j] (the table planes
  are src1 / src2, never relative);
* a source's row offsets come packed as 16-bit block offsets, four rows per 64-bit SGPR pair
  (rows 0-3, rows 4-7 of the 8-row tile); each block's tail shifts the working pair right by 16
  bits (SCC = rows left), bumps the index by 8 and jumps to the next row's block; when the pair
  is exhausted (every remaining row has c = 0: block 0 sits at offset 0) the chain leaves
  through a stub that starts the second half or ends.

Per (source, row): <= 8 full-rate VALU, 6 SALU, 1 jump (the nibble chain: <= 16 VALU, 4 SALU,
2 jumps).  Blocks are packed (variable size) -- the offsets come from the device's kGxOff
table -- so the executed table is ~24 KiB.  As in the nibble chain, a fast copy keeps the high
half of the jump target fixed and a safe copy (used only if the table straddles a 4 GiB
boundary, checked at every entry) propagates the carry.

Usage: python tools/gen_bitslice_gidx.py   (rewrites the .inc; commit the result)
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_bitslice_chain import gmul, table_planes, NPLANES  # noqa: E402

OUT = os.environ.get("NTC_GX_OUT") or os.path.join(os.path.dirname(HERE), "netcode_amd", "csrc",
                                                  "gf_bitslice_gidx.inc")
ACC = 64          # accumulator planes of row j: v[ACC + 8j .. ACC + 8j + 7]
ROWS = 8


def byte_ops(lo, hi, c):
    """acc ^= c * x on the relative accumulators v[ACC..ACC+7]: per output plane p the two
    nibbles (a_p, b_p) of row p of c's 8x8 GF(2) matrix select TL[a_p] ^ TH[b_p].  The
    accumulator is src0 and dst (the relative operands); table planes are src1 / src2."""
    cols = [gmul(c, 1 << q) for q in range(8)]
    ops = []
    for p in range(8):
        a = sum(((cols[q] >> p) & 1) << q for q in range(4))
        b = sum(((cols[4 + q] >> p) & 1) << q for q in range(4))
        acc = f"v{ACC + p}"
        if a and b:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, %[y{lo[a]}], %[y{hi[b]}] bitop3:0x96")
        elif a or b:
            ops.append(f"v_xor_b32_e64 {acc}, {acc}, %[y{lo[a] if a else hi[b]}]")
    return ops


def op_bytes(op):
    return 8          # v_bitop3_b32 and v_xor_b32_e64 are both VOP3: 8 bytes


def tail(safe, tag):
    t = ["s_lshr_b64 s[90:91], s[90:91], 16",          # next row's offset; SCC = rows left
         f"s_cbranch_scc0 Lx{tag}%=",
         "s_and_b32 s98, s90, 0xffff",
         "s_add_u32 s98, s96, s98"]
    if safe:
        t.append("s_addc_u32 s99, s97, 0")
    t += ["s_add_u32 s95, s95, 8",                      # next row: index + 8
          "s_set_gpr_idx_idx s95",
          "s_setpc_b64 s[98:99]"]
    return t


TAIL_BYTES = {False: 4 + 4 + 8 + 4 + 4 + 4 + 4, True: 4 + 4 + 8 + 4 + 4 + 4 + 4 + 4}


def layout():
    """Block offsets (bytes from the table start) for c = 0..255; block 0 (no ops) at 0.  The
    safe copy's blocks are 4 bytes longer each, so it gets its own offsets -- the fast layout is
    padded to the safe one's, and one offset table serves both."""
    lo, hi, _ = table_planes()
    off, pos = [], 0
    for c in range(256):
        off.append(pos)
        n = len(byte_ops(lo, hi, c)) * 8 + TAIL_BYTES[True]
        pos += (n + 3) // 4 * 4
    return off, pos


def dispatch_first(pair, safe, tag, empty_target):
    """Start a half: working pair = `pair`; if it holds no rows, go to `empty_target`."""
    d = [f"s_mov_b64 s[90:91], {pair}",
         "s_cmp_eq_u64 s[90:91], 0",
         f"s_cbranch_scc1 {empty_target}",
         "s_and_b32 s98, s90, 0xffff",
         "s_add_u32 s98, s96, s98"]
    if safe:
        d.append("s_addc_u32 s99, s97, 0")
    d.append("s_setpc_b64 s[98:99]")
    return d


def copy_lines(safe, off):
    tag = "s" if safe else "f"
    lo, hi, _ = table_planes()
    lines = []
    # exit stub: leaving half 0 (index < 32) starts half 1 (rows 4-7); leaving half 1 ends
    lines += [f"Lx{tag}%=:", "s_cmp_lt_u32 s95, 32", "s_cbranch_scc0 Le%=",
              "s_mov_b32 s95, 32", "s_set_gpr_idx_idx s95"]
    lines += dispatch_first("%[p1]", safe, tag, "Le%=")
    lines += [".p2align 6", f"Lt{tag}%=:"]
    for c in range(256):
        lab = f"L{tag}{c}_%="
        lines.append(f"{lab}:")
        body = byte_ops(lo, hi, c) + tail(safe, tag)
        lines += body
        nxt = off[c + 1] if c + 1 < 256 else None
        if nxt is not None:
            lines.append(f".fill {nxt - off[c]} - (. - {lab}), 1, 0")
    return lines


def chain(off, span):
    lines = ["s_mov_b32 s94, m0",                        # M0 carries the VGPR index: keep it
             "s_getpc_b64 s[96:97]", "Lg%=:",
             "s_add_u32 s96, s96, Ltf%= - Lg%=", "s_addc_u32 s97, s97, 0",
             f"s_add_u32 s98, s96, {span}", "s_cbranch_scc1 Lsafe%=",
             "s_mov_b32 s99, s97",
             "s_mov_b32 s95, 0",
             "s_set_gpr_idx_on s95, gpr_idx(SRC0,DST)"]
    lines += dispatch_first("%[p0]", False, "f", "Lxf%=")
    lines += copy_lines(False, off)
    lines += ["Lsafe%=:", "s_getpc_b64 s[96:97]", "Lh%=:",
              "s_add_u32 s96, s96, Lts%= - Lh%=", "s_addc_u32 s97, s97, 0",
              "s_mov_b32 s95, 0",
              "s_set_gpr_idx_on s95, gpr_idx(SRC0,DST)"]
    lines += dispatch_first("%[p0]", True, "s", "Lxs%=")
    lines += copy_lines(True, off)
    lines += ["Le%=:", "s_set_gpr_idx_off", "s_mov_b32 m0, s94"]
    return lines


# ---- variant 2: raw coefficient bytes, fixed 128-byte blocks, one 64-bit row register -------
# P holds the 8 rows' coefficients (row 0 in the low byte).  Block c sits at c * 128; its tail
# shifts P right by a byte (SCC = rows left, else leave), turns the new low byte into its block
# address with two shifts (no literal), advances the VGPR index by adding 8 to M0 directly
# (M0[7:0] is the index s_set_gpr_idx_on set; the mode bits sit in M0[15:12]) and jumps.
BLK2 = 128


def tail2(safe):
    t = ["s_lshr_b64 s[90:91], s[90:91], 8",           # next row's coefficient; SCC = rows left
         "s_cbranch_scc0 LQe%=",
         "s_lshl_b32 s98, s90, 24",
         "s_lshr_b32 s98, s98, 17",                      # c << 7
         "s_add_u32 s98, s96, s98"]
    if safe:
        t.append("s_addc_u32 s99, s97, 0")
    t += ["s_add_u32 m0, m0, 8",                        # next row: VGPR index + 8
          "s_setpc_b64 s[98:99]"]
    return t


def copy2(safe):
    tag = "s" if safe else "f"
    lo, hi, _ = table_planes()
    lines = [".p2align 7", f"LQu{tag}%=:"]
    for c in range(256):
        lab = f"LQv{tag}{c}_%="
        lines.append(f"{lab}:")
        lines += byte_ops(lo, hi, c) + tail2(safe)
        lines.append(f".fill {BLK2} - (. - {lab}), 1, 0")
    return lines


def chain2():
    span = 256 * BLK2
    first = ["s_mov_b64 s[90:91], %[p]",
             "s_cmp_eq_u64 s[90:91], 0", "s_cbranch_scc1 LQe%=",
             "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17",
             "s_add_u32 s98, s96, s98"]
    lines = ["s_mov_b32 s94, m0",
             "s_getpc_b64 s[96:97]", "LQg%=:",
             "s_add_u32 s96, s96, LQuf%= - LQg%=", "s_addc_u32 s97, s97, 0",
             f"s_add_u32 s98, s96, {span}", "s_cbranch_scc1 LQsafe%=",
             "s_mov_b32 s99, s97",
             "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)"]
    lines += first + ["s_setpc_b64 s[98:99]"]
    lines += copy2(False)
    lines += ["LQsafe%=:", "s_getpc_b64 s[96:97]", "LQh%=:",
              "s_add_u32 s96, s96, LQus%= - LQh%=", "s_addc_u32 s97, s97, 0",
              "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)"]
    lines += first + ["s_addc_u32 s99, s97, 0", "s_setpc_b64 s[98:99]"]
    lines += copy2(True)
    lines += ["LQe%=:", "s_set_gpr_idx_off", "s_mov_b32 m0, s94"]
    return lines


# ---- variant 3: variant 2's table ONCE, outside the kernels --------------------------------
# The 256 blocks live in a never-called holder function (ntc_gx3_tables), so the MAC loop body
# stays small (short back edge) and every kernel shares one copy.  Fixed registers: table
# planes Y[0..29] in v[Y3..Y3+29], accumulators v[ACC..ACC+63] (index-relative), s90:91 the row
# coefficients, s96:97 the table base, s92:93 the return address (s_swappc at entry).  The fast
# table keeps the jump target's high half fixed; the safe one (chosen once per kernel when the
# fast table straddles a 4 GiB boundary) propagates the carry.
Y3 = 32


def byte_ops3(lo, hi, c):
    return [op.replace("%[y", "%%[y") for op in byte_ops(lo, hi, c)]


def table3(safe):
    tag = "s" if safe else "f"
    lo, hi, _ = table_planes()
    ymap = {f"%[y{n}]": f"v{Y3 + n}" for n in range(NPLANES)}
    lines = [".p2align 7", f"ntc_gx3_{tag}:"]
    for c in range(256):
        lab = f"ntc_gx3_{tag}{c}"
        lines.append(f"{lab}:")
        body = byte_ops(lo, hi, c)
        for k, v in sorted(ymap.items(), key=lambda kv: -len(kv[0])):
            body = [b.replace(k, v) for b in body]
        t = ["s_lshr_b64 s[90:91], s[90:91], 8", f"s_cbranch_scc0 ntc_gx3_ret_{tag}",
             "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17", "s_add_u32 s98, s96, s98"]
        if safe:
            t.append("s_addc_u32 s99, s97, 0")
        t += ["s_add_u32 m0, m0, 8", "s_setpc_b64 s[98:99]"]
        lines += body + t
        lines.append(f".fill {BLK2} - (. - {lab}), 1, 0")
    lines += [f"ntc_gx3_ret_{tag}:", "s_setpc_b64 s[92:93]"]
    return lines


def main():
    off, span = layout()
    assert span < 65536, span
    lo, hi, stmts = table_planes()
    o = ["// Generated by tools/gen_bitslice_gidx.py -- do not edit by hand.",
         "// Shared-table bit-sliced GF(2^8) MAC chain, VGPR-relative rows (see the generator).",
         "#pragma once", "",
         f"constexpr int kGxAcc = {ACC};                 // first accumulator VGPR (row 0, plane 0)",
         f"constexpr uint32_t kGxSpan = {span};          // bytes of one table copy",
         "// byte offset of coefficient c's block inside the table (block 0 = no work, offset 0)",
         "__device__ constexpr uint16_t kGxOff[256] = {" + ", ".join(map(str, off)) + "};", ""]
    o.append("#define NTC_GX_CHAIN \\")
    o.append("".join(f'  "{l}\\n" \\\n' for l in chain(off, span)) + '  ""')
    o.append("")
    outs = ", ".join(f'[A{j}] "+{{v[{ACC + 8 * j}:{ACC + 8 * j + 7}]}}"(A[{j}])' for j in range(ROWS))
    o.append(f"#define NTC_GX_OUTS(A) {outs}")
    ins = ", ".join(f'[y{n}] "v"(Y[{n}])' for n in range(NPLANES))
    ins += ', [p0] "s"(P0), [p1] "s"(P1)'
    o.append(f"#define NTC_GX_INS(Y, P0, P1) {ins}")
    o.append('#define NTC_GX_CLOBBERS "s90", "s91", "s94", "s95", "s96", "s97", "s98", "s99", "scc"')
    o.append("")
    o.append("// variant 2: P = the 8 rows' coefficient bytes (row 0 lowest); fixed 128-byte blocks")
    o.append("#define NTC_GX2_CHAIN \\")
    o.append("".join(f'  "{l}\\n" \\\n' for l in chain2()) + '  ""')
    o.append('#define NTC_GX2_INS(Y, P) ' + ", ".join(f'[y{n}] "v"(Y[{n}])' for n in range(NPLANES)) +
             ', [p] "s"(P)')
    o.append('#define NTC_GX2_CLOBBERS "s90", "s91", "s94", "s96", "s97", "s98", "s99", "scc"')
    o.append("")
    o.append("// variant 3: the tables (fast, then safe) for the holder function ntc_gx3_tables")
    o.append(f"constexpr int kGx3Y = {Y3};                  // first table-plane VGPR (Y[0])")
    o.append(f"constexpr uint32_t kGx3Span = {256 * BLK2};")
    o.append("#define NTC_GX3_TABLES \\")
    o.append("".join(f'  "{l}\\n" \\\n' for l in ["s_endpgm"] + table3(False) + table3(True)) + '  ""')
    o.append('#define NTC_GX3_YPINS(Y) ' + ", ".join(f'[y{n}] "{{v{Y3 + n}}}"(Y[{n}])' for n in range(NPLANES)))
    open(OUT, "w").write("\n".join(o) + "\n")
    print("wrote", OUT, "table bytes", span)


if __name__ == "__main__":
    main()
