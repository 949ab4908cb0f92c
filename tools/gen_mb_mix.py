"""Emit tools/mb_mix.hip: do the gfx950 instruction forms that issue at half rate when a SIMD runs
only them (tools/gen_mb_issue.py: VGPR-indexed VALU, v_lshlrev by an inline constant, VALU with
an SGPR operand, taken s_setpc jumps) still cost a SIMD two slots when OTHER waves on that SIMD
issue plain VALU beside them?

Two roles share every SIMD: the blocks [0, ncu) and [2 ncu, 3 ncu) run body A, the others body B
(one block per CU per range, so each SIMD holds W/2 waves of each role).  Every wave runs its
64-instruction body `iters` times.  Reported: the span of the whole launch in shader cycles per
SIMD per (A body + B body) pair, against the two bodies run alone (the same kernel with A = B).
If A's half rate is an issue constraint of its own wave only, B's plain VALU fills the gaps and
the pair costs ~max(A, B); if it occupies the SIMD's VALU, the pair costs A + B.

Usage: python tools/gen_mb_mix.py && hipcc --offload-arch=gfx950 -O3 -w -o tools/mb_mix \
         tools/mb_mix.hip && tools/mb_mix
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_mb_issue import body, body_jump, ACC0, OPS0  # noqa: E402

BODIES = {
    "plain": lambda: body("bitop3", "cf"),
    "xor": lambda: body("xor", "cf"),
    "idx": lambda: body("bitop3", "cf", idx=True),
    "shlc": lambda: body("shl2", "cf"),
    "sgpr": lambda: body("bitop3s", "cf"),
    "tail_idx": lambda: body_jump("tail", idx=True),
    "tail": lambda: body_jump("tail", idx=False),
}
PAIRS = [("plain", "plain"), ("idx", "idx"), ("idx", "plain"), ("shlc", "shlc"), ("shlc", "plain"),
         ("sgpr", "sgpr"), ("sgpr", "plain"), ("idx", "shlc"), ("tail_idx", "tail_idx"),
         ("tail_idx", "plain"), ("tail", "plain"), ("idx", "xor")]

CLOB = ", ".join(f'"v{r}"' for r in range(ACC0, OPS0 + 32))

KERNEL = r'''
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

template <int V>
__device__ __forceinline__ void run_body(uint32_t iters)
{
  @BODIES@
}

template <int A, int B>
__global__ __launch_bounds__(256) void mb(uint32_t iters, uint32_t ncu, uint32_t* __restrict__ out)
{
  extern __shared__ uint8_t lds[];
  uint32_t seed = threadIdx.x * 0x9E3779B9u + blockIdx.x;
  asm volatile("v_mov_b32 v32, %[s]\n" @INIT@ "s_mov_b32 s40, 0x5a5a5a5a\n"
               :: [s] "v"(seed) : @CLOB@, "s40");
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  if ((blockIdx.x / ncu) & 1) run_body<B>(iters);
  else run_body<A>(iters);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
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

typedef void (*kfn)(uint32_t, uint32_t, uint32_t*);

int main()
{
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  uint32_t* out;
  (void)hipMalloc(&out, 64u << 20);
  struct Case { const char* a; const char* b; kfn fn; };
  Case cases[] = { @CASES@ };
  const int occ[] = {2, 4};
  const uint32_t iters = 4000;
  printf("{\"cus\": %d, \"insts_per_wave\": %u}\n", ncu, iters * 64);
  for (const Case& c : cases) {
    for (int W : occ) {
      const size_t lds = (160u * 1024u) / W - 1024;
      const int nb = ncu * W;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(c.fn),
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      double best = 1e30, clk = 0;
      for (int rep = 0; rep < 4; ++rep) {
        hipLaunchKernelGGL(c.fn, dim3(nb), dim3(256), lds, 0, iters, static_cast<uint32_t>(ncu), out);
        if (hipDeviceSynchronize() != hipSuccess) { printf("{\"error\": \"%s/%s\"}\n", c.a, c.b); return 1; }
        std::vector<uint32_t> h(static_cast<size_t>(nb) * 4 * 8);
        (void)hipMemcpy(h.data(), out, h.size() * 4, hipMemcpyDeviceToHost);
        std::vector<double> ck;
        uint64_t rmin = ~0ull, rmax = 0;
        for (size_t w = 0; w < static_cast<size_t>(nb) * 4; ++w) {
          const uint64_t dt = h[w * 8] | (static_cast<uint64_t>(h[w * 8 + 1]) << 32);
          const uint64_t dr = h[w * 8 + 2] | (static_cast<uint64_t>(h[w * 8 + 3]) << 32);
          const uint64_t rs = h[w * 8 + 6] | (static_cast<uint64_t>(h[w * 8 + 7]) << 32);
          rmin = std::min(rmin, rs);
          rmax = std::max(rmax, rs + dr);
          if (dr) ck.push_back(static_cast<double>(dt) / dr * 100.0);
        }
        std::sort(ck.begin(), ck.end());
        const double mhz = ck.empty() ? 0 : ck[ck.size() / 2];
        const double span_cyc = static_cast<double>(rmax - rmin) / 100.0 * mhz;
        // per SIMD: W/2 waves of each role, each `iters` bodies -> cycles per (A + B) body pair
        const double v = span_cyc / (W / 2.0) / iters;
        if (rep > 0 && v < best) { best = v; clk = mhz; }
      }
      printf("{\"a\": \"%s\", \"b\": \"%s\", \"W\": %d, \"cyc_per_body_pair_per_simd\": %.1f, \"clock_mhz\": %.0f}\n",
             c.a, c.b, W, best, clk);
      fflush(stdout);
    }
  }
  return 0;
}
'''


def main():
    init = "".join(f'"v_add_u32 v{r}, {r * 7 + 1}, v32\\n" ' for r in range(ACC0 + 1, OPS0 + 32))
    names = list(BODIES)
    bodies = []
    for i, n in enumerate(names):
        asm = "".join(f'"{l}\\n" ' for l in BODIES[n]())
        bodies.append(
            f'if constexpr (V == {i}) asm volatile("s_mov_b32 s41, %[n]\\n" "L{i}_%=:\\n" {asm}'
            f'"s_sub_u32 s41, s41, 1\\n" "s_cmp_lg_u32 s41, 0\\n" "s_cbranch_scc1 L{i}_%=\\n" '
            f':: [n] "s"(iters) : {CLOB}, "s40", "s41", "s50", "s51", "s52", "s53", "s54", "m0", "scc");')
    cases = [f'{{"{a}", "{b}", mb<{names.index(a)}, {names.index(b)}>}}' for a, b in PAIRS]
    src = (KERNEL.replace("@INIT@", init).replace("@CLOB@", CLOB)
           .replace("@BODIES@", "\n  ".join(bodies)).replace("@CASES@", ", ".join(cases)))
    open(os.path.join(HERE, "mb_mix.hip"), "w").write(src)
    print("wrote tools/mb_mix.hip")


if __name__ == "__main__":
    main()
