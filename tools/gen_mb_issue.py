"""Emit tools/mb_issue.hip: VALU issue rate of the bit-sliced MAC's instruction forms on gfx950.

Round-5 question: the round-3 chain microbenchmark (tools/gen_microbench_chain.py) measured
8 plain v_bitop3 per row at 25.3 SIMD cycles (3.2 per instruction) at 4 waves/SIMD -- not the
2 cycles a wave64 VALU op takes on a SIMD-32 -- and VGPR-indexed ones at 4.9.  Its operands
were picked without regard to VGPR banks (register number mod 4).  Here every variant is a
64-instruction straight-line body with 32 independent accumulators, looped in asm, and the
operand banks are controlled:
  cf    : the three source VGPRs of every instruction sit in three different banks
  b2    : two of the three sources share a bank
  same  : all three sources in one bank
Forms: v_bitop3_b32 (XOR3), v_xor_b32_e32, v_fma_f32 (control), the same under
s_set_gpr_idx_on (SRC0,DST), v_bitop3 with an SGPR operand, and scalar ops (alone and
alternating with plain VALU in one wave: the decode plan's selector arithmetic).  Each wave stamps s_memtime /
s_memrealtime around its loop (vector stores only), so cycles per instruction per SIMD =
shader cycles / (waves per SIMD x instructions per wave), at the clock the chip actually held.

Usage: python tools/gen_mb_issue.py && hipcc --offload-arch=gfx950 -O3 -o tools/mb_issue \
         tools/mb_issue.hip && tools/mb_issue
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ACC0 = 32          # accumulators v32..v63 (32 of them)
OPS0 = 64          # operands v64..v95


def acc(i):
    return ACC0 + i


def body(form, banks, idx=False):
    """64 instructions; accumulator i % 32 updated twice per body."""
    out = []
    if idx:
        out.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
    for n in range(64):
        a = acc(n % 32)
        ba = a % 4
        # choose operand registers by bank pattern relative to the accumulator's bank
        if banks == "cf":
            b1, b2 = (ba + 1) % 4, (ba + 2) % 4
        elif banks == "b2":
            b1, b2 = (ba + 1) % 4, (ba + 1) % 4
        else:  # same
            b1, b2 = ba, ba
        base = (n * 3) % 8          # spread over v64..v95 (8 regs per bank)
        o1 = OPS0 + 4 * base + b1
        o2 = OPS0 + 4 * ((base + 3) % 8) + b2
        if form == "bitop3":
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{o1}, v{o2} bitop3:0x96")
        elif form == "xor":
            out.append(f"v_xor_b32_e32 v{a}, v{o1}, v{a}")
        elif form == "xor64":       # VOP3 encoding of the 2-input XOR
            out.append(f"v_xor_b32_e64 v{a}, v{a}, v{o1}")
        elif form == "fma":
            out.append(f"v_fma_f32 v{a}, v{o1}, v{o2}, v{a}")
        elif form == "bitop3s":
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{o1}, s40 bitop3:0x96")
        elif form == "perm":
            out.append(f"v_perm_b32 v{a}, v{o1}, v{o2}, v{a}")
        elif form == "xors":          # VOP2 with an SGPR src0
            out.append(f"v_xor_b32_e32 v{a}, s40, v{a}")
        elif form == "shl3":          # VOP3 shift with an inline-constant operand
            out.append(f"v_lshlrev_b32_e64 v{a}, 4, v{o1}")
        elif form == "shl2":          # VOP2 shift with an inline-constant operand
            out.append(f"v_lshlrev_b32_e32 v{a}, 4, v{o1}")
        elif form == "lshl64":        # 64-bit shift of an even-aligned pair
            d = ACC0 + 2 * (n % 16)
            out.append(f"v_lshlrev_b64 v[{d}:{d + 1}], 4, v[{OPS0 + 2 * (n % 16)}:{OPS0 + 2 * (n % 16) + 1}]")
        elif form == "lshr32v":       # 32-bit shift with the amount in a VGPR
            out.append(f"v_lshrrev_b32_e32 v{a}, v{o2}, v{o1}")
        elif form == "add":
            out.append(f"v_add_u32_e32 v{a}, v{o1}, v{a}")
        elif form == "alignbit":
            out.append(f"v_alignbit_b32 v{a}, v{o1}, v{o2}, 4")
        elif form == "lshlor":
            out.append(f"v_lshl_or_b32 v{a}, v{o1}, 4, v{o2}")
        elif form == "bfi":
            out.append(f"v_bfi_b32 v{a}, v{o1}, v{o2}, v{a}")
        elif form == "cndmask":
            out.append(f"v_cndmask_b32_e32 v{a}, v{o1}, v{o2}, vcc")
        elif form == "mov":
            out.append(f"v_mov_b32_e32 v{a}, v{o1}")
        elif form == "mul24":
            out.append(f"v_mul_u32_u24_e32 v{a}, v{o1}, v{o2}")
        elif form == "lshladd64":     # gfx950 v_lshl_add_u64
            d = ACC0 + 2 * (n % 16)
            out.append(f"v_lshl_add_u64 v[{d}:{d + 1}], v[{OPS0 + 2 * (n % 16)}:{OPS0 + 2 * (n % 16) + 1}], 1, v[{d}:{d + 1}]")
        elif form == "andlit":        # VOP2 with a literal src0
            out.append(f"v_and_b32_e32 v{a}, 0x0f0f0f0f, v{o1}")
        elif form == "addc0":         # VOP2 with an inline-constant src0
            out.append(f"v_add_u32_e32 v{a}, 4, v{o1}")
        elif form == "shrc1":         # VOP3 shift: VGPR amount, inline-constant value (src1)
            out.append(f"v_lshrrev_b32_e64 v{a}, v{o1}, 64")
        elif form == "bitop3c0":      # bitop3 with an inline constant in src0
            out.append(f"v_bitop3_b32 v{a}, 7, v{o1}, v{a} bitop3:0x96")
        elif form == "bitop3c1":      # bitop3 with an inline constant in src1
            out.append(f"v_bitop3_b32 v{a}, v{a}, 7, v{o1} bitop3:0x96")
        elif form == "readlane":
            out.append(f"v_readlane_b32 s{42 + n % 8}, v{o1}, {n % 64}")
        elif form == "salu_lit":      # scalar AND with a literal (the plan's selector masks)
            out.append(f"s_and_b32 s{42 + n % 8}, s{42 + (n + 3) % 8}, 0x7070707")
        elif form == "salu_ss":       # scalar XOR of two SGPRs
            out.append(f"s_xor_b32 s{42 + n % 8}, s{42 + n % 8}, s{42 + (n + 1) % 8}")
        elif form == "salu_valu":     # one scalar and one plain VALU op alternating (same wave)
            if n % 2:
                out.append(f"s_xor_b32 s{42 + n % 8}, s{42 + n % 8}, s{42 + (n + 1) % 8}")
            else:
                out.append(f"v_bitop3_b32 v{a}, v{a}, v{o1}, v{o2} bitop3:0x96")
        elif form == "bitop3c":       # bitop3 with an inline-constant operand
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{o1}, 7 bitop3:0x96")
    if idx:
        out.append("s_set_gpr_idx_off")
    return out


def body_jump(kind, idx=False):
    """64 bitop3 (banks cf) in 8 blocks of 8, each block ended by a taken jump to the next one:
    kind 'br' = s_branch, 'setpc' = s_getpc / s_add / s_setpc (the chain's form), 'tail' = the
    chain's 7-SALU tail shape with a PC-relative s_setpc; idx: under s_set_gpr_idx_on with
    M0 += 8 per block (the chain's row step, wrapping over the 4 row blocks v32..v63)."""
    ops = body("bitop3", "cf")
    out = []
    if idx:
        out.append("s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)")
    for blk in range(8):
        blk_ops = []
        for n in range(8):
            o = ops[blk * 8 + n]
            if idx:   # row 0's registers (v32..v39) in every block; M0 selects the row
                a = ACC0 + n
                parts = o.split()
                o = f"v_bitop3_b32 v{a}, v{a}, {parts[3]} {parts[4]} bitop3:0x96"
            blk_ops.append(o)
        out += blk_ops
        if kind == "br":
            out.append(f"s_branch LJ{blk}_%=")
        elif kind == "setpc":
            out += [f"s_getpc_b64 s[50:51]", f"LG{blk}_%=:",
                    f"s_add_u32 s50, s50, LJ{blk}_%= - LG{blk}_%=",
                    "s_addc_u32 s51, s51, 0", "s_setpc_b64 s[50:51]"]
        elif kind == "tail":
            out += ["s_lshr_b64 s[52:53], s[52:53], 8", "s_lshl_b32 s54, s52, 24",
                    "s_lshr_b32 s54, s54, 17", f"s_getpc_b64 s[50:51]", f"LG{blk}_%=:",
                    f"s_add_u32 s50, s50, LJ{blk}_%= - LG{blk}_%=", "s_addc_u32 s51, s51, 0",
                    "s_setpc_b64 s[50:51]"]
        if idx and kind != "none":
            out.insert(len(out) - 1, "s_add_u32 m0, m0, 8" if blk % 4 != 3 else "s_sub_u32 m0, m0, 24")
        elif idx:
            out.append("s_add_u32 m0, m0, 8" if blk % 4 != 3 else "s_sub_u32 m0, m0, 24")
        out.append(f"LJ{blk}_%=:")
    if idx:
        out.append("s_set_gpr_idx_off")
    return out


LACC, LOPS, LADDR = 32, 96, 128     # lane-chain layout: 8 rows of accumulators, operands, addresses


def body_lanechain(idx):
    """8 blocks (rows) per loop; block j: v_readlane s98 <- lane M0 (=8j) of v128 (the address of
    block j+1; lane 56 = the end label), 8 bitop3 on row j (accumulator in SRC2: gpr_idx(SRC2,DST)
    with M0 = 8j, or absolute row-0 registers without indexing), s_add m0 8, s_setpc s[98:99]."""
    ops = body("bitop3", "cf")
    # the blocks' s_setpc keeps the high dword of s_getpc: skip the test if the code straddles a
    # 4 GiB boundary (LEND is the highest label), so no jump can leave the function
    pre = ["s_getpc_b64 s[50:51]", "LPC_%=:", "s_add_u32 s52, s50, LEND_%= - LPC_%=",
           "s_addc_u32 s53, s51, 0", "s_cmp_eq_u32 s53, s51", "s_cbranch_scc0 LSKIP_%=",
           "v_mov_b32 v128, s52"]
    for j in range(7):
        pre += [f"s_add_u32 s52, s50, LB{j + 1}_%= - LPC_%=", f"v_writelane_b32 v128, s52, {8 * j}"]
    pre += ["s_add_u32 s60, s50, LB0_%= - LPC_%=", "s_mov_b32 s61, s51", "s_mov_b32 s99, s51", "s_nop 4"]
    loop = ["LLOOP_%=:"]
    loop.append("s_set_gpr_idx_on 0, gpr_idx(SRC2,DST)" if idx else "s_mov_b32 m0, 0")
    loop.append("s_setpc_b64 s[60:61]")
    for j in range(8):
        loop.append(f"LB{j}_%=:")
        loop.append("v_readlane_b32 s98, v128, m0")
        for n in range(8):
            parts = ops[j * 8 + n].replace(",", "").split()
            o1 = LOPS + int(parts[3][1:]) - OPS0
            o2 = LOPS + int(parts[4][1:]) - OPS0
            a = LACC + n if idx else LACC + 8 * j + n
            loop.append(f"v_bitop3_b32 v{a}, v{o1}, v{o2}, v{a} bitop3:0x96")
        loop.append("s_add_u32 m0, m0, 8")
        loop.append("s_setpc_b64 s[98:99]")
    loop.append("LEND_%=:")
    if idx:
        loop.append("s_set_gpr_idx_off")
    return pre, loop


VARIANTS = [
    ("bitop3_cf", "bitop3", "cf", False),
    ("bitop3_b2", "bitop3", "b2", False),
    ("bitop3_same", "bitop3", "same", False),
    ("xor_cf", "xor", "cf", False),
    ("xor_same", "xor", "same", False),
    ("xor64_cf", "xor64", "cf", False),
    ("fma_cf", "fma", "cf", False),
    ("fma_same", "fma", "same", False),
    ("bitop3s_cf", "bitop3s", "cf", False),
    ("perm_cf", "perm", "cf", False),
    ("idx_bitop3_cf", "bitop3", "cf", True),
    ("idx_bitop3_same", "bitop3", "same", True),
    ("idx_xor_cf", "xor", "cf", True),
    ("rows_idx", "jump:none", "cf", True),
    ("jump_br", "jump:br", "cf", False),
    ("jump_setpc", "jump:setpc", "cf", False),
    ("jump_tail", "jump:tail", "cf", False),
    ("jump_tail_idx", "jump:tail", "cf", True),
    ("lshl64", "lshl64", "cf", False),
    ("lshr32v", "lshr32v", "cf", False),
    ("add", "add", "cf", False),
    ("alignbit", "alignbit", "cf", False),
    ("lshlor", "lshlor", "cf", False),
    ("bfi", "bfi", "cf", False),
    ("cndmask", "cndmask", "cf", False),
    ("mov", "mov", "cf", False),
    ("mul24", "mul24", "cf", False),
    ("lshladd64", "lshladd64", "cf", False),
    ("andlit", "andlit", "cf", False),
    ("addc0", "addc0", "cf", False),
    ("shrc1", "shrc1", "cf", False),
    ("bitop3c0", "bitop3c0", "cf", False),
    ("bitop3c1", "bitop3c1", "cf", False),
    ("readlane", "readlane", "cf", False),
    ("xors_cf", "xors", "cf", False),
    ("shl3_c", "shl3", "cf", False),
    ("shl2_c", "shl2", "cf", False),
    ("bitop3c", "bitop3c", "cf", False),
    ("salu_lit", "salu_lit", "cf", False),
    ("salu_ss", "salu_ss", "cf", False),
    ("salu_valu", "salu_valu", "cf", False),
    ("lanechain_noidx", "lane", "cf", False),
    ("lanechain_idx", "lane", "cf", True),
]

CLOB = ", ".join(f'"v{r}"' for r in range(ACC0, OPS0 + 32))

KERNEL = r'''
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

template <int V>
__global__ __launch_bounds__(256) void mb(uint32_t iters, uint32_t* __restrict__ out)
{
  extern __shared__ uint8_t lds[];
  uint32_t seed = threadIdx.x * 0x9E3779B9u + blockIdx.x;
  uint64_t t0, t1, r0, r1;
  asm volatile(
      "v_mov_b32 v32, %[s]\n" @INIT@
      "s_mov_b32 s40, 0x5a5a5a5a\n"
      :: [s] "v"(seed) : @CLOB@, "s40");
  t0 = __builtin_amdgcn_s_memtime();
  r0 = __builtin_amdgcn_s_memrealtime();
  @BODIES@
  t1 = __builtin_amdgcn_s_memtime();
  r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x;
  asm volatile("v_xor_b32 %0, v32, v33\n" "v_xor_b32 %0, %0, v63\n" : "=v"(x) :: @CLOB@);
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t* o = out + (blockIdx.x * 4u + wave) * 8u;
  if (lane < 4) {
    const uint64_t v = lane == 0 ? t1 - t0 : lane == 1 ? r1 - r0 : lane == 2 ? x + lds[0] : r0;
    o[2 * lane] = static_cast<uint32_t>(v);
    o[2 * lane + 1] = static_cast<uint32_t>(v >> 32);
  }
}

typedef void (*kfn)(uint32_t, uint32_t*);

int main()
{
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  uint32_t* out;
  (void)hipMalloc(&out, 64u << 20);
  struct Case { const char* name; kfn fn; };
  Case cases[] = { @CASES@ };
  const int occ[] = {1, 2, 3, 4};
  const uint32_t iters = 4000;
  printf("{\"cus\": %d, \"clock_khz\": %d, \"insts_per_wave\": %u}\n", ncu, prop.clockRate, iters * 64);
  for (const Case& c : cases) {
    for (int W : occ) {
      const size_t lds = (160u * 1024u) / W - 1024;    // W blocks of 4 waves per CU = W waves/SIMD
      const int nb = ncu * W;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(c.fn),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      double best = 1e30, clk = 0, wavec = 0;
      for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(c.fn, dim3(nb), dim3(256), lds, 0, iters, out);
        if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s\"}\n", c.name); return 1; }
        std::vector<uint32_t> h(static_cast<size_t>(nb) * 4 * 8);
        (void)hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
        std::vector<double> ck;
        uint64_t rmin = ~0ull, rmax = 0;
        double wcyc = 0;
        for (size_t w = 0; w < static_cast<size_t>(nb) * 4; ++w) {
          const uint64_t dt = h[w * 8] | (static_cast<uint64_t>(h[w * 8 + 1]) << 32);
          const uint64_t dr = h[w * 8 + 2] | (static_cast<uint64_t>(h[w * 8 + 3]) << 32);
          const uint64_t rs = h[w * 8 + 6] | (static_cast<uint64_t>(h[w * 8 + 7]) << 32);
          rmin = std::min(rmin, rs);
          rmax = std::max(rmax, rs + dr);
          wcyc += static_cast<double>(dt);
          if (dr) ck.push_back(static_cast<double>(dt) / dr * 100.0);   // MHz
        }
        std::sort(ck.begin(), ck.end());
        const double mhz = ck.empty() ? 0 : ck[ck.size() / 2];
        // the span from the first wave's start to the last wave's end, in shader cycles at the
        // median clock, per SIMD-instruction: span * (SIMDs) / (all instructions)
        const double span_cyc = static_cast<double>(rmax - rmin) / 100.0 * mhz;
        const double total = static_cast<double>(nb) * 4 * iters * 64;
        const double v = span_cyc * ncu * 4 / total;
        if (rep > 0 && v < best) { best = v; clk = mhz; wavec = wcyc / (nb * 4.0) / (iters * 64.0); }
      }
      printf("{\"case\": \"%s\", \"W\": %d, \"cyc_per_inst_per_simd\": %.3f, \"wave_cyc_per_inst\": %.3f, \"clock_mhz\": %.0f}\n",
             c.name, W, best, wavec, clk);
      fflush(stdout);
    }
  }
  return 0;
}
'''


def main():
    init = "".join(f'"v_add_u32 v{r}, {r * 7 + 1}, v32\\n" ' for r in range(ACC0 + 1, OPS0 + 32))
    bodies = []
    cases = []
    for i, (name, form, banks, idx) in enumerate(VARIANTS):
        q = lambda ls: "".join(f'"{l}\\n" ' for l in ls)
        if form == "lane":
            pre, loop = body_lanechain(idx)
            clob = ", ".join(f'"v{r}"' for r in range(LACC, LADDR + 1))
            bodies.append(
                f'if constexpr (V == {i}) asm volatile("s_mov_b32 s41, %[n]\\n" {q(pre)} {q(loop)}'
                f'"s_sub_u32 s41, s41, 1\\n" "s_cmp_lg_u32 s41, 0\\n" "s_cbranch_scc1 LLOOP_%=\\n" "LSKIP_%=:\\n" '
                f':: [n] "s"(iters) : {clob}, "s40", "s41", "s50", "s51", "s52", "s53", "s60", "s61", "s98", "s99", "m0", "scc");')
            cases.append(f'{{"{name}", mb<{i}>}}')
            continue
        lines = body_jump(form[5:], idx) if form.startswith("jump:") else body(form, banks, idx)
        asm = q(lines)
        bodies.append(
            f'if constexpr (V == {i}) asm volatile("s_mov_b32 s41, %[n]\\n" "L{i}_%=:\\n" {asm}'
            f'"s_sub_u32 s41, s41, 1\\n" "s_cmp_lg_u32 s41, 0\\n" "s_cbranch_scc1 L{i}_%=\\n" '
            f':: [n] "s"(iters) : {CLOB}, "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "m0", "scc");')
        cases.append(f'{{"{name}", mb<{i}>}}')
    src = (KERNEL.replace("@INIT@", init).replace("@CLOB@", CLOB)
           .replace("@BODIES@", "\n  ".join(bodies)).replace("@CASES@", ", ".join(cases)))
    open(os.path.join(HERE, "mb_issue.hip"), "w").write(src)
    print("wrote tools/mb_issue.hip")


if __name__ == "__main__":
    main()
