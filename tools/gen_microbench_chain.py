"""Emit tools/microbench_chain.hip: what bounds the shared-table bit-sliced MAC chain on gfx950.

The MAC spends ~60 % of its instruction bytes in a chain of jumps into one table of 256 blocks
(block c = the <= 8 v_bitop3 of acc ^= c*x on the row's 8 accumulator planes, then a scalar tail
that finds the next row's block and jumps).  Each wave here runs only that chain, on random
nonzero coefficients read like the product reads them (s_load of 8 bytes per 8 rows), with
optional straight-line filler VALU standing in for the per-source transpose and plane tables.

Variants (per row):
  0 straight : 8 v_bitop3 into absolute accumulators, no jump (VALU + issue ceiling)
  1 product  : 128-byte blocks, 7-SALU tail (shift, exit branch, 2 shifts, add, M0 += 8, setpc)
  2 nobranch : 6-SALU tail (no exit branch: after the last row the zero byte selects block 0,
               which returns)
  3 half     : the product tail with 4 v_bitop3 per block (blocks fit 2 fetch lines, not 3)
  4 noidx    : the product chain without VGPR-relative addressing (every row hits row 0)
  5 spaced   : the product tail, blocks 256 bytes apart (64 KiB table)
R = 8 or 16 rows per chain (R = 16: two chain calls per iteration, accumulators v64..v191).
Occupancy W waves per SIMD is set by dynamic LDS (one 256-thread block per W on every CU).

Usage: python tools/gen_microbench_chain.py && hipcc --offload-arch=gfx950 -O3 \
         -o tools/microbench_chain tools/microbench_chain.hip && tools/microbench_chain
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_bitslice_table import table_planes, NPLANES, gmul  # noqa: E402

def byte_ops3(lo, hi, c):
    """acc ^= c * x on v64..v71 (plane operands as %%[yN] placeholders)."""
    cols = [gmul(c, 1 << q) for q in range(8)]
    ops = []
    for p in range(8):
        a = sum(((cols[q] >> p) & 1) << q for q in range(4))
        b = sum(((cols[4 + q] >> p) & 1) << q for q in range(4))
        acc = f"v{64 + p}"
        if a and b:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, %%[y{lo[a]}], %%[y{hi[b]}] bitop3:0x96")
        elif a or b:
            ops.append(f"v_xor_b32_e64 {acc}, {acc}, %%[y{lo[a] if a else hi[b]}]")
    return ops


Y0 = 32          # table planes v32..v61
Y0W = 2          # wide variant: planes of group 0 v2..v31, group 1 v32..v61
ACC = 64         # accumulators: row j plane p = v[64 + 8j + p]


def body(c, half=False):
    lo, hi, _ = table_planes()
    ops = [o.replace("%%[y", "%[y") for o in byte_ops3(lo, hi, c)]
    out = []
    for o in ops:
        for n in sorted(range(NPLANES), key=lambda n: -len(str(n))):
            o = o.replace(f"%[y{n}]", f"v{Y0 + n}")
        out.append(o)
    return out[:4] if half else out


def tail(v, tag):
    if v == 2:
        return ["s_lshr_b64 s[90:91], s[90:91], 8", "s_lshl_b32 s98, s90, 24",
                "s_lshr_b32 s98, s98, 17", "s_add_u32 s98, s96, s98", "s_add_u32 m0, m0, 8",
                "s_setpc_b64 s[98:99]"]
    sh = 16 if v == 5 else 17
    return ["s_lshr_b64 s[90:91], s[90:91], 8", f"s_cbranch_scc0 mb{tag}_ret",
            "s_lshl_b32 s98, s90, 24", f"s_lshr_b32 s98, s98, {sh}", "s_add_u32 s98, s96, s98",
            "s_add_u32 m0, m0, 8", "s_setpc_b64 s[98:99]"]


def wide_body(c):
    lo, hi, _ = table_planes()
    ops = [o.replace("%%[y", "%[y") for o in byte_ops3(lo, hi, c)]
    out = []
    for g in range(2):                 # group g: accumulators v64+8g.., planes Y0W + 30g ..
        for o in ops:
            for n in sorted(range(NPLANES), key=lambda n: -len(str(n))):
                o = o.replace(f"%[y{n}]", f"v{Y0W + 30 * g + n}")
            for p in range(8):
                o = o.replace(f"v{ACC + p},", f"v{ACC + 8 * g + p},")
            out.append(o)
    return out


def rowtab(ntab):
    """ntab per-row tables (absolute accumulators of row j), 32 KiB each, contiguous; row j's
    block jumps into table (j+1) % ntab."""
    tag = f"rt{ntab}"
    lines = ["s_endpgm", ".p2align 15", f"mb{tag}_t:"]
    for j in range(ntab):
        for c in range(256):
            lab = f"mb{tag}_{j}_{c}"
            lines.append(f"{lab}:")
            ops = []
            for o in body(c):
                for p_ in range(8):
                    o = o.replace(f"v{ACC + p_},", f"v{ACC + 8 * j + p_},")
                ops.append(o)
            step = 32768 if j + 1 < ntab else -32768 * (ntab - 1)
            if c == 0:              # nonzero coefficients: byte 0 past the last row = return
                lines += ["s_setpc_b64 s[92:93]", f".fill 128 - (. - {lab}), 1, 0"]
                continue
            lines += ops + ["s_lshr_b64 s[90:91], s[90:91], 8",
                            "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17",
                            f"s_add_u32 s96, s96, {step & 0xFFFFFFFF}", "s_add_u32 s98, s96, s98",
                            "s_setpc_b64 s[98:99]"]
            lines.append(f".fill 128 - (. - {lab}), 1, 0")
    return lines


def table12():
    lo, hi, _ = table_planes()
    lines = ["s_endpgm", ".p2align 7", "mbv12_t:"]
    for c in range(256):
        lab = f"mbv12_{c}"
        lines.append(f"{lab}:")
        for o in [o.replace("%%[y", "%[y") for o in byte_ops3(lo, hi, c)]:
            for n in sorted(range(NPLANES), key=lambda n: -len(str(n))):
                o = o.replace(f"%[y{n}]", f"v{2 + n}")
            for p_ in range(8):
                o = o.replace(f"v{ACC + p_},", f"v{32 + p_},")
            lines.append(o)
        lines += ["s_lshr_b64 s[90:91], s[90:91], 8", "s_cbranch_scc0 mbv12_ret",
                  "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 17", "s_add_u32 s98, s96, s98",
                  "s_add_u32 m0, m0, 8", "s_setpc_b64 s[98:99]"]
        lines.append(f".fill 128 - (. - {lab}), 1, 0")
    lines += ["mbv12_ret:", "s_setpc_b64 s[92:93]"]
    return lines


def table(v):
    if v == 6:
        tag = "v6"
        lines = ["s_endpgm", ".p2align 8", "mbv6_t:"]
        for c in range(256):
            lab = f"mbv6_{c}"
            lines.append(f"{lab}:")
            lines += wide_body(c) + ["s_lshr_b64 s[90:91], s[90:91], 8", "s_cbranch_scc0 mbv6_ret",
                                     "s_lshl_b32 s98, s90, 24", "s_lshr_b32 s98, s98, 16",
                                     "s_add_u32 s98, s96, s98", "s_add_u32 m0, m0, 16",
                                     "s_setpc_b64 s[98:99]"]
            lines.append(f".fill 256 - (. - {lab}), 1, 0")
        lines += ["mbv6_ret:", "s_setpc_b64 s[92:93]"]
        return lines, 256
    blk = 256 if v == 5 else 128
    tag = f"v{v}"
    lines = ["s_endpgm", f".p2align {8 if blk == 256 else 7}", f"mb{tag}_t:"]
    for c in range(256):
        lab = f"mb{tag}_{c}"
        lines.append(f"{lab}:")
        if v == 2 and c == 0:
            lines.append("s_setpc_b64 s[92:93]")
        else:
            lines += body(c, half=(v == 3)) + tail(v, tag)
        lines.append(f".fill {blk} - (. - {lab}), 1, 0")
    lines += [f"mb{tag}_ret:", "s_setpc_b64 s[92:93]"]
    return lines, blk


def asm_str(lines):
    return "".join(f'    "{l}\\n"\n' for l in lines)


def main():
    o = ['// Generated by tools/gen_microbench_chain.py -- do not edit.',
         '#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdlib>',
         '#include <cstdint>', '#include <vector>', '',
         'typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));', '']
    spans = {}
    for v in (1, 2, 3, 4, 5, 6):
        if v == 4:
            continue                         # variant 4 reuses variant 1's table
        lines, blk = table(v)
        spans[v] = 256 * blk
        o.append(f'extern "C" __device__ __attribute__((used, noinline)) void mb_tab{v}() {{ asm volatile(\n'
                 + asm_str(lines) + '  ); }')
    spans[4] = spans[1]
    o.append('extern "C" __device__ __attribute__((used, noinline)) void mb_tab12() { asm volatile(\n'
             + asm_str(table12()) + '  ); }')
    o.append('#define MB_OUTS12(A) ' + ", ".join(f'[A{j}] "+{{v[{32 + 8 * j}:{32 + 8 * j + 7}]}}"(A[{j}])' for j in range(16)))
    o.append('#define MB_YINS12(Y) ' + ", ".join(f'[y{n}] "{{v{2 + n}}}"(Y[{n}])' for n in range(NPLANES)))
    for nf in (70,):
        fill = []
        for i in range(nf):
            a, b = 160 + i % 6, 160 + (i + 3) % 6
            fill.append(f"v_bitop3_b32 v{a}, v{a}, v{b}, v{2 + i % 30} bitop3:0x96" if i % 3 == 0
                        else f"v_xor_b32 v{a}, v{b}, v{a}")
        o.append(f'#define MB_FILL{nf}_160 \\\n' + "".join(f'  "{l}\\n" \\\n' for l in fill) + '  ""')
    for nt in (2, 8):
        o.append(f'extern "C" __device__ __attribute__((used, noinline)) void mb_rowtab{nt}() {{ asm volatile(\n'
                 + asm_str(rowtab(nt)) + '  ); }')
    outs = ", ".join(f'[A{j}] "+{{v[{ACC + 8 * j}:{ACC + 8 * j + 7}]}}"(A[{j}])' for j in range(16))
    yins = ", ".join(f'[y{n}] "{{v{Y0 + n}}}"(Y[{n}])' for n in range(NPLANES))
    o.append(f'#define MB_OUTS(A) {outs}')
    o.append(f'#define MB_OUTS8(A) ' + ", ".join(f'[A{j}] "+{{v[{ACC + 8 * j}:{ACC + 8 * j + 7}]}}"(A[{j}])' for j in range(8)))
    o.append(f'#define MB_YINS(Y) {yins}')
    o.append('#define MB_YINSW(Y) ' + ", ".join(f'[y{n}] "{{v{Y0W + n}}}"(Y[{n}])' for n in range(60)))
    # straight-line stand-in: row j plane p = acc ^ Y[a] ^ Y[b], fixed pattern
    st = []
    for j in range(8):
        for p in range(8):
            st.append(f"v_bitop3_b32 v{ACC + 8 * j + p}, v{ACC + 8 * j + p}, v{Y0 + (j + p) % 15}, "
                      f"v{Y0 + 15 + (3 * j + p) % 15} bitop3:0x96")
    o.append('#define MB_STRAIGHT \\\n' + "".join(f'  "{l}\\n" \\\n' for l in st) + '  ""')
    # operand-slot variants of the indexed straight line (M0 += 8 per row): 20 SRC2+DST,
    # 21 SRC1+DST, 22 DST only, 23 SRC0 only, 24 VOP2 v_xor SRC0+DST (2 ops per plane)
    slot = {20: ("SRC2,DST", "v{a}, v{y1}, v{y2}, v{a}"), 21: ("SRC1,DST", "v{a}, v{y1}, v{a}, v{y2}"),
            22: ("DST", "v{a}, v{y1}, v{y2}, v{b}"), 23: ("SRC0", "v{b}, v{a}, v{y1}, v{y2}")}
    for v in (20, 21, 22, 23, 24):
        mode = "SRC0,DST" if v == 24 else slot[v][0]
        st2 = [f"s_set_gpr_idx_on 0, gpr_idx({mode})"]
        for j in range(8):
            for p_ in range(8):
                y1, y2 = Y0 + (j + p_) % 15, Y0 + 15 + (3 * j + p_) % 15
                if v == 24:
                    st2.append(f"v_xor_b32 v{ACC + p_}, v{ACC + p_}, v{y1}")
                else:
                    ops = slot[v][1].format(a=ACC + p_, b=16 + p_, y1=y1, y2=y2)
                    st2.append(f"v_bitop3_b32 {ops} bitop3:0x96")
            st2.append("s_add_u32 m0, m0, 8")
        st2.append("s_set_gpr_idx_off")
        o.append(f'#define MB_STRAIGHT_IDX{v} \\\n' + "".join(f'  "{l}\\n" \\\n' for l in st2) + '  ""')
    # the same ops on row 0's registers, VGPR-indexed; M0 += 8 after each row (variant 9) or not (8)
    for v in (8, 9):
        st2 = ["s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)"]
        for j in range(8):
            for p_ in range(8):
                st2.append(f"v_bitop3_b32 v{ACC + p_}, v{ACC + p_}, v{Y0 + (j + p_) % 15}, "
                           f"v{Y0 + 15 + (3 * j + p_) % 15} bitop3:0x96")
            if v == 9:
                st2.append("s_add_u32 m0, m0, 8")
        st2.append("s_set_gpr_idx_off")
        o.append(f'#define MB_STRAIGHT_IDX{v} \\\n' + "".join(f'  "{l}\\n" \\\n' for l in st2) + '  ""')
    for nf, base in ((17, 16), (35, 16), (70, 16), (35, 192), (140, 192)):
        fill = []
        for i in range(nf):
            a, b = base + i % 8, base + (i + 3) % 8
            fill.append(f"v_bitop3_b32 v{a}, v{a}, v{b}, v{Y0 + i % 30} bitop3:0x96" if i % 3 == 0
                        else f"v_xor_b32 v{a}, v{b}, v{a}")
        o.append(f'#define MB_FILL{nf}_{base} \\\n' + "".join(f'  "{l}\\n" \\\n' for l in fill) + '  ""')
    o.append('')
    o.append(KERNEL.replace("@SPAN1@", str(spans[1])).replace("@SPAN2@", str(spans[2]))
             .replace("@SPAN3@", str(spans[3])).replace("@SPAN5@", str(spans[5])))
    open(os.path.join(HERE, "microbench_chain.hip"), "w").write("\n".join(o) + "\n")
    print("wrote tools/microbench_chain.hip")


KERNEL = r'''
// table base of variant V (PC-relative); returns 0 if the table straddles a 4 GiB boundary
template <int V>
__device__ __forceinline__ uint64_t table_base()
{
  uint64_t b;
  uint32_t bad;
#define MB_BASE(SYM, SPAN) asm volatile("s_getpc_b64 s[96:97]\n" \
      "s_add_u32 s96, s96, " SYM "@rel32@lo+4\n" "s_addc_u32 s97, s97, " SYM "@rel32@hi+12\n" \
      "s_add_u32 s98, s96, " #SPAN "\n" "s_cselect_b32 %1, 1, 0\n" "s_mov_b64 %0, s[96:97]\n" \
      : "=s"(b), "=s"(bad) :: "s96", "s97", "s98", "scc")
  if constexpr (V == 1 || V == 4 || V == 7) MB_BASE("mbv1_t", @SPAN1@);
  else if constexpr (V == 2) MB_BASE("mbv2_t", @SPAN2@);
  else if constexpr (V == 3) MB_BASE("mbv3_t", @SPAN3@);
  else if constexpr (V == 5) MB_BASE("mbv5_t", @SPAN5@);
  else if constexpr (V == 12) MB_BASE("mbv12_t", 32768);
  else if constexpr (V == 10) MB_BASE("mbrt8_t", 262144);
  else if constexpr (V == 11) MB_BASE("mbrt2_t", 65536);
  else MB_BASE("mbv6_t", 65536);
  return bad ? 0 : b;
}

template <int V, int R>
__device__ __forceinline__ void chain(u32x8 (&A)[16], const uint32_t (&Y)[60], uint64_t P, uint64_t tb,
                                      uint32_t idx0)
{
  constexpr int SH = V == 5 ? 16 : 17;
  if constexpr (V != 4 && R == 8) {
    asm volatile("s_mov_b32 s94, m0\n"
                 "s_set_gpr_idx_on %[i0], gpr_idx(SRC0,DST)\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, %[sh]\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_set_gpr_idx_off\n"
                 "s_mov_b32 m0, s94\n"
                 : MB_OUTS8(A), [p] "+{s[90:91]}"(P)
                 : MB_YINS(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0), [sh] "i"(SH)
                 : "s92", "s93", "s94", "s98", "s99", "scc");
  } else if constexpr (V == 6) {
    asm volatile("s_mov_b32 s94, m0\n"
                 "s_set_gpr_idx_on %[i0], gpr_idx(SRC0,DST)\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 16\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_set_gpr_idx_off\n"
                 "s_mov_b32 m0, s94\n"
                 : MB_OUTS(A), [p] "+{s[90:91]}"(P)
                 : MB_YINSW(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0)
                 : "s92", "s93", "s94", "s98", "s99", "scc");
  } else if constexpr (V == 7) {
    // gpr-index mode stays on for the whole kernel (index 0 outside the chain)
#define MB_PERSIST(OUTS) asm volatile("s_set_gpr_idx_idx %[i0]\n" \
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 17\n" \
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n" \
                 "s_swappc_b64 s[92:93], s[98:99]\n" \
                 "s_set_gpr_idx_idx 0\n" \
                 : OUTS(A), [p] "+{s[90:91]}"(P) \
                 : MB_YINS(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0) \
                 : "s92", "s93", "s98", "s99", "scc")
    if constexpr (R == 8) MB_PERSIST(MB_OUTS8);
    else MB_PERSIST(MB_OUTS);
  } else if constexpr (V == 12) {
    asm volatile("s_mov_b32 s94, m0\n"
                 "s_set_gpr_idx_on %[i0], gpr_idx(SRC0,DST)\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 17\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_set_gpr_idx_off\n"
                 "s_mov_b32 m0, s94\n"
                 : MB_OUTS12(A), [p] "+{s[90:91]}"(P)
                 : MB_YINS12(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0)
                 : "s92", "s93", "s94", "s98", "s99", "scc");
  } else if constexpr (V == 10 || V == 11) {
    asm volatile("s_mov_b64 s[88:89], s[96:97]\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 17\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_mov_b64 s[96:97], s[88:89]\n"
                 : MB_OUTS8(A), [p] "+{s[90:91]}"(P)
                 : MB_YINS(Y), [tb] "{s[96:97]}"(tb)
                 : "s88", "s89", "s92", "s93", "s98", "s99", "scc");
  } else if constexpr (V == 4) {
    asm volatile("s_mov_b32 s94, m0\n"
                 "s_mov_b32 m0, %[i0]\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, 17\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_mov_b32 m0, s94\n"
                 : MB_OUTS8(A), [p] "+{s[90:91]}"(P)
                 : MB_YINS(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0)
                 : "s92", "s93", "s94", "s98", "s99", "scc");
  } else {
    asm volatile("s_mov_b32 s94, m0\n"
                 "s_set_gpr_idx_on %[i0], gpr_idx(SRC0,DST)\n"
                 "s_lshl_b32 s98, s90, 24\n" "s_lshr_b32 s98, s98, %[sh]\n"
                 "s_add_u32 s98, s96, s98\n" "s_mov_b32 s99, s97\n"
                 "s_swappc_b64 s[92:93], s[98:99]\n"
                 "s_set_gpr_idx_off\n"
                 "s_mov_b32 m0, s94\n"
                 : MB_OUTS(A), [p] "+{s[90:91]}"(P)
                 : MB_YINS(Y), [tb] "{s[96:97]}"(tb), [i0] "s"(idx0), [sh] "i"(SH)
                 : "s92", "s93", "s94", "s98", "s99", "scc");
  }
}

template <int V, int R, int F>
__global__ __launch_bounds__(256) void mb(const uint64_t* __restrict__ coef, uint32_t iters,
                                          uint32_t* __restrict__ out)
{
  extern __shared__ uint8_t lds[];
  u32x8 A[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) A[j] = u32x8{0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t Y[60];
#pragma unroll
  for (int n = 0; n < 60; ++n) Y[n] = threadIdx.x * 0x9E3779B9u + n * 0x85EBCA6Bu;
  uint64_t tb = 0;
  if constexpr (V != 0) {
    tb = table_base<V>();
    if (!tb) { if (threadIdx.x == 0) out[blockIdx.x] = 0xDEAD; return; }
  }
  if constexpr (V == 7) asm volatile("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)" ::: "memory");
  const uint32_t wave = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
  const uint64_t* cp = coef + (wave * 7u) % 4096u * 2u;
  for (uint32_t it = 0; it < iters; ++it) {
    const auto* cq = reinterpret_cast<const __attribute__((address_space(4))) uint64_t*>(
        reinterpret_cast<uintptr_t>(cp));
    const uint64_t P0 = cq[0];
    const uint64_t P1 = cq[1];
    cp = cp + 2 >= coef + 8192 ? coef : cp + 2;
#define MB_CLOB "v192", "v193", "v194", "v195", "v196", "v197", "v198", "v199"
#define MB_CLOB16 "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23"
    if constexpr (V == 12) {
      if constexpr (F == 70) asm volatile(MB_FILL70_160 ::: "v160", "v161", "v162", "v163", "v164", "v165");
    } else if constexpr (V == 6) {
      if constexpr (F == 35) asm volatile(MB_FILL35_192 ::: MB_CLOB);
      if constexpr (F == 140) asm volatile(MB_FILL140_192 ::: MB_CLOB);
    } else {
      if constexpr (F == 17) asm volatile(MB_FILL17_16 ::: MB_CLOB16);
      if constexpr (F == 35) asm volatile(MB_FILL35_16 ::: MB_CLOB16);
      if constexpr (F == 70) asm volatile(MB_FILL70_16 ::: MB_CLOB16);
    }
    if constexpr (V >= 20 && V <= 24) {
#define MB_SIDX(N) asm volatile("s_mov_b32 s94, m0\n" MB_STRAIGHT_IDX##N "s_mov_b32 m0, s94" : MB_OUTS8(A) : MB_YINS(Y), "s"(P0) : "s94", "scc", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23")
      if constexpr (V == 20) MB_SIDX(20);
      if constexpr (V == 21) MB_SIDX(21);
      if constexpr (V == 22) MB_SIDX(22);
      if constexpr (V == 23) MB_SIDX(23);
      if constexpr (V == 24) MB_SIDX(24);
    } else if constexpr (V == 8 || V == 9) {
      if constexpr (V == 8) asm volatile("s_mov_b32 s94, m0\n" MB_STRAIGHT_IDX8 "s_mov_b32 m0, s94" : MB_OUTS8(A) : MB_YINS(Y), "s"(P0) : "s94", "scc");
      else asm volatile("s_mov_b32 s94, m0\n" MB_STRAIGHT_IDX9 "s_mov_b32 m0, s94" : MB_OUTS8(A) : MB_YINS(Y), "s"(P0) : "s94", "scc");
    } else if constexpr (V == 0) {
      if constexpr (R == 8) {
        asm volatile(MB_STRAIGHT : MB_OUTS8(A) : MB_YINS(Y), "s"(P0));
      } else {
        asm volatile(MB_STRAIGHT : MB_OUTS(A) : MB_YINS(Y), "s"(P0));
        asm volatile(MB_STRAIGHT : MB_OUTS(A) : MB_YINS(Y), "s"(P1));
      }
    } else {
      chain<V, R>(A, Y, P0, tb, 0);
      if constexpr (R == 16 && V != 6) chain<V, R>(A, Y, P1, tb, V == 4 ? 0 : 64);
    }
  }
  if constexpr (V == 7) asm volatile("s_set_gpr_idx_off" ::: "memory");
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < R; ++j)
#pragma unroll
    for (int p = 0; p < 8; ++p) x ^= A[j][p];
  out[blockIdx.x * 256 + threadIdx.x] = x + lds[0];
}

typedef void (*kfn)(const uint64_t*, uint32_t, uint32_t*);

template <int V, int R, int F> kfn K() { return mb<V, R, F>; }

int main(int argc, char** argv)
{
  int ncu = 256;
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  ncu = prop.multiProcessorCount;
  std::vector<uint64_t> h(8192);
  uint64_t s = 88172645463325252ull;
  for (auto& x : h) {
    uint64_t v = 0;
    for (int b = 0; b < 8; ++b) {
      s ^= s << 13; s ^= s >> 7; s ^= s << 17;
      v |= static_cast<uint64_t>(1 + s % 255) << (8 * b);   // nonzero coefficients
    }
    x = v;
  }
  uint64_t* d;
  uint32_t* out;
  (void)hipMalloc(&d, h.size() * 8);
  (void)hipMalloc(&out, 64u << 20);
  (void)hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  struct Case { const char* name; int v, r, f; kfn fn; };
  Case cases[] = {
    // wide: 8 rows x 64 B per lane (counted as 16 wave-rows of 32 B); fill per 64 B source = 140
    {"straight", 0, 8, 0, K<0, 8, 0>()}, {"idx_src0_dst", 9, 8, 0, K<9, 8, 0>()},
    {"idx_src2_dst", 20, 8, 0, K<20, 8, 0>()}, {"idx_src1_dst", 21, 8, 0, K<21, 8, 0>()},
    {"idx_dst_only", 22, 8, 0, K<22, 8, 0>()}, {"idx_src0_only", 23, 8, 0, K<23, 8, 0>()},
    {"idx_vop2_xor", 24, 8, 0, K<24, 8, 0>()},
  };
  Case old_cases[] = {
    {"straight", 0, 8, 0, K<0, 8, 0>()}, {"straight", 0, 16, 0, K<0, 16, 0>()},
    {"product", 1, 8, 0, K<1, 8, 0>()}, {"product", 1, 16, 0, K<1, 16, 0>()},
    {"nobranch", 2, 8, 0, K<2, 8, 0>()}, {"nobranch", 2, 16, 0, K<2, 16, 0>()},
    {"half", 3, 8, 0, K<3, 8, 0>()}, {"half", 3, 16, 0, K<3, 16, 0>()},
    {"noidx", 4, 8, 0, K<4, 8, 0>()},
    {"spaced", 5, 8, 0, K<5, 8, 0>()},
  };
  (void)old_cases;
  const int occ[] = {1, 2, 3, 4, 6, 8};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("{\"cus\": %d, \"clock_khz\": %d}\n", ncu, prop.clockRate);
  for (const Case& c : cases) {
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(c.fn));
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(c.fn),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int W : occ) {
      const int maxw = 512 / ((fa.numRegs + 7) / 8 * 8);
      if (W > maxw) continue;
      const size_t lds = (160 * 1024) / W - 1024;
      const uint32_t iters = c.r == 16 ? 10000 : 20000;
      const int blocks = ncu * W;
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(c.fn, dim3(blocks), dim3(256), lds, 0, d, iters, out);
        if (hipGetLastError() != hipSuccess) { printf("launch error\n"); return 1; }
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) { printf("launch failed\n"); return 1; }
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      uint32_t flag = 0;
      (void)hipMemcpy(&flag, out, 4, hipMemcpyDeviceToHost);
      const double rows = static_cast<double>(blocks) * 4 * iters * c.r;   // wave-rows
      // one wave-row = 8 bitop3 x 64 lanes x 32 bits = 2048 byte-MACs
      const double tmac = rows * 2048 / (best * 1e-3) / 1e12;
      // cycles per wave-row per SIMD at the nominal clock
      const double cyc = best * 1e-3 * 2.4e9 / (rows / (4.0 * ncu));
      printf("{\"case\": \"%s\", \"R\": %d, \"W\": %d, \"vgprs\": %d, \"ms\": %.3f, \"Tbytemac_s\": %.1f, "
             "\"cyc_per_row_per_simd_2g4\": %.2f, \"bad\": %d}\n",
             c.name, c.r, W, fa.numRegs, best, tmac, cyc, flag == 0xDEAD);
      fflush(stdout);
    }
  }
  return 0;
}
'''

if __name__ == "__main__":
    main()
