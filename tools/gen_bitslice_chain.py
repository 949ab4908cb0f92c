"""Generate netcode_amd/csrc/gf_bitslice_chain.inc — the jump-chained bit-sliced MAC block tables.

Bit-sliced GF(2^8) multiply-accumulate: a lane holds 32 bytes as 8 bit-planes
x_0..x_7.  Multiplication by a constant m is GF(2)-linear: plane p of m*x is the XOR of the input
planes q whose bit p of m*alpha^q is set.  Four-Russians split: per source the 15 non-empty XOR
combinations of planes 0-3 (TL) and of planes 4-7 (TH) are built once (22 XORs; singletons are the
planes themselves), 30 distinct planes Y[0..29] in all; then every output plane of m*x is
TL[a_p] ^ TH[b_p] -- one 3-input v_bitop3 (or one v_xor when a half is empty).

For a row tile of R rows one source contributes to 2R "sites" (row j, coefficient nibble h): the
low nibble multiplies x by v, the high nibble by v*alpha^4 (c*x = lo(c)*x ^ hi(c)*(alpha^4 x)).
Each site owns 16 blocks (one per nibble value v) of at most 8 ops that XOR into the row's 8
accumulator planes, then jump to the next site's block: the per-source dispatch is a chain of
2R `s_setpc_b64`, with the block offsets of every (source, site) precomputed on the device
(`bj_offsets` kernel: offset = site * kBjSite + kBjVo[v]).  `.fill` pads every block to exactly
its table size, so an encoding that grew would be an assembler error, never a silent misjump.
(Full 256-entry Four-Russians blocks per row would halve the ops again, but 8 rows x 20 KiB of
code thrash the instruction cache: tools/gen_microbench_fr.py.)

Two copies of the tables share one asm statement and one layout: the fast chain keeps the high
half of the jump target fixed (s_add + s_setpc per site); if the fast tables straddle a 4 GiB
boundary (checked at each chain entry, never seen in practice) the safe copy, whose tails also
propagate the carry, runs instead.

Usage: python tools/gen_bitslice_chain.py   (rewrites the .inc; commit the result)
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("NTC_BJ_OUT") or os.path.join(os.path.dirname(HERE), "netcode_amd", "csrc",
                                                 "gf_bitslice_chain.inc")
TILES = (16, 8, 4)


NPLANES = 30


def gmul(a, b):
    """GF(2^8) product, polynomial 0x11D."""
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


def nibble_ops(lo, hi, m, j):
    """acc[j] ^= m * x: per output plane p, TL[a_p] ^ TH[b_p] with (a_p, b_p) the two nibbles of
    row p of m's 8x8 GF(2) matrix (column q = m * alpha^q)."""
    cols = [gmul(m, 1 << q) for q in range(8)]
    ops = []
    for p in range(8):
        a = sum(((cols[q] >> p) & 1) << q for q in range(4))
        b = sum(((cols[4 + q] >> p) & 1) << q for q in range(4))
        acc = f"%[a{j}_{p}]"
        if a and b:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, %[y{lo[a]}], %[y{hi[b]}] bitop3:0x96")
        elif a or b:
            ops.append(f"v_xor_b32_e32 {acc}, %[y{lo[a] if a else hi[b]}], {acc}")
    return ops


def block_bytes(ops):
    return sum(8 if o.startswith("v_bitop3") else 4 for o in ops)


def block_body(planes, j, h, v):
    lo, hi = planes
    if v == 0:
        return []
    return nibble_ops(lo, hi, v if h == 0 else gmul(v, 16), j)


TAIL = 12      # s_add [+ s_addc] + s_setpc
ALIGN = int(os.environ.get("NTC_BJ_ALIGN", "16"))   # every block starts ALIGN-byte aligned


def _sizes():
    lo, hi, _ = table_planes()
    need = [0] * 16
    for h in range(2):
        for v in range(16):
            need[v] = max(need[v], block_bytes(block_body((lo, hi), 0, h, v)))
    return [(n + TAIL + ALIGN - 1) // ALIGN * ALIGN for n in need]


SIZES = _sizes()
VO = [sum(SIZES[:v]) for v in range(16)]
SITE = sum(SIZES)


def tables(y, R, safe):
    """2R sites x 16 blocks; fast and safe tables share one layout (block v of site s at
    s * SITE + VO[v]), so the same precomputed offsets address either."""
    tag = "s" if safe else "f"
    lines = []
    nsites = 2 * R
    for site in range(nsites):
        j, h = divmod(site, 2)
        for v in range(16):
            lab = f"L{tag}{site}_{v}_%="
            lines.append(f"{lab}:")
            lines += block_body(y, j, h, v)
            if site + 1 < nsites:
                lines.append(f"s_add_u32 s98, s96, %[o{site + 1}]")
                if safe:
                    lines.append("s_addc_u32 s99, s97, 0")
                lines.append("s_setpc_b64 s[98:99]")
            else:
                lines.append("s_branch Le%=")
            lines.append(f".fill {SIZES[v]} - (. - {lab}), 1, 0")
    return lines


def chain_lines(y, R):
    span = 2 * R * SITE
    # NTC_BJ_EXTRA_SALU=n (timing experiment only): n dummy scalar ops per chain entry
    extra = ["s_add_u32 s96, s96, 0"] * int(os.environ.get("NTC_BJ_EXTRA_SALU", "0"))
    lines = ["s_getpc_b64 s[96:97]", "Lg%=:",
             "s_add_u32 s96, s96, Ltf%= - Lg%=", "s_addc_u32 s97, s97, 0"] + extra + [

             # fast path iff [Ltf, Ltf + span) does not cross a 4 GiB boundary
             f"s_add_u32 s98, s96, {span}", "s_cbranch_scc1 Lsafe%=",
             "s_mov_b32 s99, s97",
             "s_add_u32 s98, s96, %[o0]",
             "s_setpc_b64 s[98:99]", ".p2align 6", "Ltf%=:"]
    lines += tables(y, R, safe=False)
    lines += ["Lsafe%=:", "s_getpc_b64 s[96:97]", "Lh%=:",
              "s_add_u32 s96, s96, Lts%= - Lh%=", "s_addc_u32 s97, s97, 0",
              "s_add_u32 s98, s96, %[o0]", "s_addc_u32 s99, s97, 0",
              "s_setpc_b64 s[98:99]", ".p2align 6", "Lts%=:"]
    lines += tables(y, R, safe=True)
    lines.append("Le%=:")
    return lines


def main():
    lo, hi, stmts = table_planes()
    y = (lo, hi)
    o = ["// Generated by tools/gen_bitslice_chain.py -- do not edit by hand.",
         "// Jump-chained bit-sliced GF(2^8) MAC blocks (see the generator's docstring).",
         "#pragma once", "",
         f"constexpr uint32_t kBjSite = {SITE};          // bytes per site (16 nibble blocks)",
         "// byte offset of nibble value v's block inside a site",
         "__device__ constexpr uint32_t kBjVo[16] = {" + ", ".join(map(str, VO)) + "};",
         f"constexpr int kBjPlanes = {NPLANES};                   // input planes + their XOR combinations", "",
         "// Y[8..29]: the XOR combinations of input planes 0-3 and 4-7 (Four-Russians tables).",
         "#define NTC_BJ_TABLES(Y) \\"]
    o += [f"  {st} \\" for st in stmts]
    o.append("")
    for R in TILES:
        o.append(f"#define NTC_BJ_CHAIN_R{R} \\")
        o.append("".join(f'  "{l}\\n" \\\n' for l in chain_lines(y, R)) + '  ""')
        o.append("")
        outs = ", ".join(f'[a{j}_{p}] "+v"(A[{j}][{p}])' for j in range(R) for p in range(8))
        o.append(f"#define NTC_BJ_OUTS_R{R}(A) {outs}")
        ins = ", ".join(f'[y{n}] "v"(Y[{n}])' for n in range(NPLANES))
        ins += ", " + ", ".join(f'[o{s}] "s"(O[{s}])' for s in range(2 * R))
        o.append(f"#define NTC_BJ_INS_R{R}(Y, O) {ins}")
        o.append("")
    o.append('#define NTC_BJ_CLOBBERS "s96", "s97", "s98", "s99", "scc"')
    open(OUT, "w").write("\n".join(o) + "\n")
    print("wrote", OUT, "site bytes", SITE)


if __name__ == "__main__":
    main()
