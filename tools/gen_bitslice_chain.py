"""Generate netcode_amd/csrc/gf_bitslice_chain.inc — the jump-chained bit-sliced MAC block tables.

Bit-sliced GF(2^8) multiply-accumulate: a lane holds 32 bytes as 8 bit-planes
x_0..x_7; y_t = alpha^t * x (t = 0..7) are 8-plane values built by the xtime recurrence for the
field polynomial 0x11D (x^8 = x^4 + x^3 + x^2 + 1), so only 3 planes per step are new: 29
distinct planes Y[0..28] in all.  c * x = XOR_{t in bits(c)} y_t.

For a row tile of R rows one source contributes to 2R "sites" (row j, coefficient nibble h).
Each site owns 16 blocks (one per nibble value v) that XOR the selected y planes into the row's
8 accumulator planes, then jump to the next site's block: the per-source dispatch is a chain of
2R `s_setpc_b64`, with the block offsets of every (source, site) precomputed on the device
(`bj_offsets` kernel: offset = site * kBjSite + kBjVo[v]).  Block sizes depend only on popcount(v)
(8 VOP2 or VOP3 per XOR round); `.fill` pads every block to exactly its table size, so an
encoding that grew would be an assembler error, never a silent misjump.

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


def popcount(v):
    return bin(v).count("1")


def valu_bytes(v):
    return {0: 0, 1: 32, 2: 64, 3: 96, 4: 128}[popcount(v)]


TAIL = 12      # s_add [+ s_addc] + s_setpc
ALIGN = int(os.environ.get("NTC_BJ_ALIGN", "16"))   # every block starts ALIGN-byte aligned
SIZES = [(valu_bytes(v) + TAIL + ALIGN - 1) // ALIGN * ALIGN for v in range(16)]
VO = [sum(SIZES[:v]) for v in range(16)]
SITE = sum(SIZES)


def xtime_planes():
    """y[t][p] -> index into the distinct-plane list Y, plus the C++ statements that build Y."""
    y = [list(range(8))]
    stmts, n = [], 8
    for t in range(1, 8):
        u = y[-1]
        nxt = [u[7], u[0], None, None, None, u[4], u[5], u[6]]
        for p, src in ((2, 1), (3, 2), (4, 3)):
            stmts.append(f"Y[{n}] = Y[{u[src]}] ^ Y[{u[7]}];")
            nxt[p] = n
            n += 1
        y.append(nxt)
    assert n == 29
    return y, stmts


def block_body(y, j, h, v):
    """Instructions for acc[j] ^= sum_{t in bits(v)} y[4h + t], interleaved across planes."""
    ts = [4 * h + t for t in range(4) if v >> t & 1]
    rounds = []
    for p in range(8):
        regs = [f"%[y{y[t][p]}]" for t in ts]
        acc = f"%[a{j}_{p}]"
        ops = []
        if len(regs) == 1:
            ops.append(f"v_xor_b32_e32 {acc}, {regs[0]}, {acc}")
        elif len(regs) >= 2:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, {regs[0]}, {regs[1]} bitop3:0x96")
            if len(regs) == 3:
                ops.append(f"v_xor_b32_e32 {acc}, {regs[2]}, {acc}")
            elif len(regs) == 4:
                ops.append(f"v_bitop3_b32 {acc}, {acc}, {regs[2]}, {regs[3]} bitop3:0x96")
        rounds.append(ops)
    out = []
    for k in range(2):                       # first op of every plane, then the second ones
        out += [r[k] for r in rounds if len(r) > k]
    return out


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
    lines = ["s_getpc_b64 s[96:97]", "Lg%=:",
             "s_add_u32 s96, s96, Ltf%= - Lg%=", "s_addc_u32 s97, s97, 0",
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
    y, stmts = xtime_planes()
    o = ["// Generated by tools/gen_bitslice_chain.py -- do not edit by hand.",
         "// Jump-chained bit-sliced GF(2^8) MAC blocks (see the generator's docstring).",
         "#pragma once", "",
         f"constexpr uint32_t kBjSite = {SITE};          // bytes per site (16 nibble blocks)",
         "// byte offset of nibble value v's block inside a site",
         "__device__ constexpr uint32_t kBjVo[16] = {" + ", ".join(map(str, VO)) + "};",
         "constexpr int kBjPlanes = 29;                   // distinct planes of y_0..y_7", "",
         "// Y[8..28] from the bit-planes Y[0..7]: y_t = alpha^t x for the polynomial 0x11D.",
         "#define NTC_BJ_XTIME(Y) \\"]
    o += [f"  {st} \\" for st in stmts]
    o.append("")
    for R in TILES:
        o.append(f"#define NTC_BJ_CHAIN_R{R} \\")
        o.append("".join(f'  "{l}\\n" \\\n' for l in chain_lines(y, R)) + '  ""')
        o.append("")
        outs = ", ".join(f'[a{j}_{p}] "+v"(A[{j}][{p}])' for j in range(R) for p in range(8))
        o.append(f"#define NTC_BJ_OUTS_R{R}(A) {outs}")
        ins = ", ".join(f'[y{n}] "v"(Y[{n}])' for n in range(29))
        ins += ", " + ", ".join(f'[o{s}] "s"(O[{s}])' for s in range(2 * R))
        o.append(f"#define NTC_BJ_INS_R{R}(Y, O) {ins}")
        o.append("")
    o.append('#define NTC_BJ_CLOBBERS "s96", "s97", "s98", "s99", "scc"')
    open(OUT, "w").write("\n".join(o) + "\n")
    print("wrote", OUT, "site bytes", SITE)


if __name__ == "__main__":
    main()
