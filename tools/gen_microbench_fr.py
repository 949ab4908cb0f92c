"""Emit tools/microbench_fr.hip: cost of a Four-Russians jump chain for the bit-sliced GF(2^8) MAC.

Per (source, row) the MAC needs acc[j][p] ^= T_lo[a_p(c)] ^ T_hi[b_p(c)] for the 8 output planes
p, where T_lo / T_hi are the 16 XOR combinations of input planes 0-3 / 4-7 and (a_p, b_p) the two
nibbles of row p of the 8x8 GF(2) matrix of c.  One block per (row slot, c): 8 v_bitop3 + a
chained jump, fixed 80-byte blocks.  The code is row slots x 20 KiB, so the question measured here
is what the instruction cache does to a dispatch when every wave jumps to random blocks.

Modes: 0 straight-line 8 bitop3 per row (VALU ceiling), 1 chain with random coefficients,
2 chain with one coefficient for all waves (every block fetch hits the same lines).
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
BLK = 80


def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def nibbles(c):
    """(a_p, b_p) for p = 0..7: bit q of a_p = bit p of c*alpha^q (q < 4), b_p likewise (q >= 4)."""
    cols = [gmul(c, 1 << q) for q in range(8)]
    out = []
    for p in range(8):
        a = sum(((cols[q] >> p) & 1) << q for q in range(4))
        b = sum(((cols[4 + q] >> p) & 1) << q for q in range(4))
        out.append((a, b))
    return out


def block(j, c, nxt):
    ops = []
    for p, (a, b) in enumerate(nibbles(c)):
        acc = f"%[a{j}_{p}]"
        if a and b:
            ops.append(f"v_bitop3_b32 {acc}, {acc}, %[l{a}], %[h{b}] bitop3:0x96")
        elif a:
            ops.append(f"v_xor_b32_e64 {acc}, %[l{a}], {acc}")
        elif b:
            ops.append(f"v_xor_b32_e64 {acc}, %[h{b}], {acc}")
    ops += nxt
    return ops


def chain(R):
    s = ["s_getpc_b64 s[96:97]", "Lg%=:", "s_add_u32 s96, s96, Lt%= - Lg%=",
         "s_addc_u32 s97, s97, 0", "s_mov_b32 s99, s97", "s_add_u32 s98, s96, %[o0]",
         "s_setpc_b64 s[98:99]", ".p2align 7", "Lt%=:"]
    for j in range(R):
        nxt = ([f"s_add_u32 s98, s96, %[o{j + 1}]", "s_setpc_b64 s[98:99]"] if j + 1 < R
               else ["s_branch Le%="])
        for c in range(256):
            lab = f"L{j}_{c}_%="
            s.append(f"{lab}:")
            s += block(j, c, nxt)
            s.append(f".fill {BLK} - (. - {lab}), 1, 0")
    s.append("Le%=:")
    body = "".join(f'"{l}\\n"\n' for l in s)
    outs = ", ".join(f'[a{j}_{p}] "+v"(acc[{j}][{p}])' for j in range(R) for p in range(8))
    ins = ", ".join(f'[l{v}] "v"(T[{v}])' for v in range(1, 16))
    ins += ", " + ", ".join(f'[h{v}] "v"(T[{16 + v}])' for v in range(1, 16))
    ins += ", " + ", ".join(f'[o{j}] "s"(o[{j}])' for j in range(R))
    return f"asm volatile(\n{body}: {outs}\n: {ins}\n: \"s96\", \"s97\", \"s98\", \"s99\", \"scc\");"


def gidx_chain(R):
    """One shared table of 256 blocks on the accumulators v[100:107]; each row stub sets the VGPR
    index (SRC0 + DST relative, M0 = 8j) and calls the block with s_swappc; the block returns."""
    s = ["s_mov_b32 s94, m0", "s_getpc_b64 s[96:97]", "Lg%=:", "s_add_u32 s96, s96, Lt%= - Lg%=",
         "s_addc_u32 s97, s97, 0", "s_mov_b32 s99, s97"]
    for j in range(R):
        s += [f"s_set_gpr_idx_on %[m{j}], gpr_idx(SRC0,DST)", f"s_add_u32 s98, s96, %[o{j}]",
              "s_swappc_b64 s[92:93], s[98:99]", "s_set_gpr_idx_off"]
    s += ["s_branch Le%=", ".p2align 7", "Lt%=:"]
    for c in range(256):
        lab = f"L{c}_%="
        s.append(f"{lab}:")
        ops = []
        for p, (a, b) in enumerate(nibbles(c)):
            acc = f"v{100 + p}"
            if a and b:
                ops.append(f"v_bitop3_b32 {acc}, {acc}, %[l{a}], %[h{b}] bitop3:0x96")
            elif a:
                ops.append(f"v_xor_b32_e64 {acc}, {acc}, %[l{a}]")
            elif b:
                ops.append(f"v_xor_b32_e64 {acc}, {acc}, %[h{b}]")
        s += ops + ["s_setpc_b64 s[92:93]", f".fill {BLK} - (. - {lab}), 1, 0"]
    s += ["Le%=:", "s_mov_b32 m0, s94"]
    body = "".join(f'"{l}\\n"\n' for l in s)
    outs = ", ".join(f'[A{j}] "+{{v[{100 + 8 * j}:{107 + 8 * j}]}}"(A[{j}])' for j in range(R))
    ins = ", ".join(f'[l{v}] "v"(T[{v}])' for v in range(1, 16))
    ins += ", " + ", ".join(f'[h{v}] "v"(T[{16 + v}])' for v in range(1, 16))
    ins += ", " + ", ".join(f'[o{j}] "s"(o[{j}])' for j in range(R))
    ins += ", " + ", ".join(f'[m{j}] "s"({8 * j}u)' for j in range(R))
    return (f"asm volatile(\n{body}: {outs}\n: {ins}\n"
            ": \"s96\", \"s97\", \"s98\", \"s99\", \"s92\", \"s93\", \"s94\", \"scc\", \"memory\");")


def straight(R):
    lines = []
    for j in range(R):
        for p in range(8):
            lines.append(f'"v_bitop3_b32 %[a{j}_{p}], %[a{j}_{p}], %[l{1 + (p + j) % 15}], %[h{1 + (3 * p + j) % 15}] bitop3:0x96\\n"')
    outs = ", ".join(f'[a{j}_{p}] "+v"(acc[{j}][{p}])' for j in range(R) for p in range(8))
    ins = ", ".join(f'[l{v}] "v"(T[{v}])' for v in range(1, 16))
    ins += ", " + ", ".join(f'[h{v}] "v"(T[{16 + v}])' for v in range(1, 16))
    return "asm volatile(\n" + "\n".join(lines) + f"\n: {outs}\n: {ins});"


SRC = r'''// Generated by tools/gen_microbench_fr.py -- Four-Russians jump-chain microbenchmark (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int R, int MODE>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed, int iters)
{
  uint32_t acc[R][8], T[32];
  for (int j = 0; j < R; ++j)
    for (int p = 0; p < 8; ++p) acc[j][p] = seed ^ (threadIdx.x * (p + 3 + j));
  for (int v = 0; v < 32; ++v) T[v] = seed * (v + 7) + threadIdx.x;
  uint32_t lcg = __builtin_amdgcn_readfirstlane(seed + (MODE == 2 ? 0u : blockIdx.x * 977u + (threadIdx.x >> 6) * 131u));
  for (int i = 0; i < iters; ++i) {
    // per "source": rebuild the tables (22 XORs, as the real kernel would)
#pragma unroll
    for (int v = 3; v < 16; ++v) if (v & (v - 1)) T[v] = T[v & (v - 1)] ^ T[v & -v];
#pragma unroll
    for (int v = 3; v < 16; ++v) if (v & (v - 1)) T[16 + v] = T[16 + (v & (v - 1))] ^ T[16 + (v & -v)];
    if constexpr (MODE == 0) {
      BODY0
    } else {
      uint32_t o[R];
#pragma unroll
      for (int j = 0; j < R; ++j) {
        if (MODE == 1) lcg = lcg * 1664525u + 1013904223u;
        o[j] = __builtin_amdgcn_readfirstlane(j * 256u * BLKB + ((lcg >> 12) & 255u) * BLKB);
      }
      BODY1
    }
    T[1] ^= acc[0][0]; T[17] ^= acc[R - 1][7];
  }
  uint32_t r = 0;
  for (int j = 0; j < R; ++j)
    for (int p = 0; p < 8; ++p) r ^= acc[j][p];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef uint32_t v8u __attribute__((ext_vector_type(8)));
template <int R>
__global__ __launch_bounds__(256) void kern3(uint32_t* out, uint32_t seed, int iters)
{
  v8u A[R];
  uint32_t T[32];
  for (int j = 0; j < R; ++j)
    for (int p = 0; p < 8; ++p) A[j][p] = seed ^ (threadIdx.x * (p + 3 + j));
  for (int v = 0; v < 32; ++v) T[v] = seed * (v + 7) + threadIdx.x;
  uint32_t lcg = __builtin_amdgcn_readfirstlane(seed + blockIdx.x * 977u + (threadIdx.x >> 6) * 131u);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int v = 3; v < 16; ++v) if (v & (v - 1)) T[v] = T[v & (v - 1)] ^ T[v & -v];
#pragma unroll
    for (int v = 3; v < 16; ++v) if (v & (v - 1)) T[16 + v] = T[16 + (v & (v - 1))] ^ T[16 + (v & -v)];
    uint32_t o[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      lcg = lcg * 1664525u + 1013904223u;
      o[j] = __builtin_amdgcn_readfirstlane(((lcg >> 12) & 255u) * BLKB);
    }
    BODY3
    T[1] ^= A[0][0]; T[17] ^= A[R - 1][7];
  }
  uint32_t r = 0;
  for (int j = 0; j < R; ++j)
    for (int p = 0; p < 8; ++p) r ^= A[j][p];
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int R>
double run3(uint32_t* d, int blocks, int iters)
{
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern3<R><<<blocks, 256>>>(d, 1, iters);
  (void)hipEventRecord(e0);
  kern3<R><<<blocks, 256>>>(d, 1, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e6 / iters;
}

template <int R, int MODE>
double run(uint32_t* d, int blocks, int iters)
{
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kern<R, MODE><<<blocks, 256>>>(d, 1, iters);
  (void)hipEventRecord(e0);
  kern<R, MODE><<<blocks, 256>>>(d, 1, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e6 / iters;
}

template <int R>
void sweep(uint32_t* d, int cus)
{
  {  // shared-table gpr-index chain must compute what the per-slot chain computes
    const int n = cus * 256;
    uint32_t *h1 = new uint32_t[n], *h2 = new uint32_t[n];
    kern<R, 1><<<cus, 256>>>(d, 5, 37);
    (void)hipMemcpy(h1, d, n * 4, hipMemcpyDeviceToHost);
    kern3<R><<<cus, 256>>>(d, 5, 37);
    (void)hipMemcpy(h2, d, n * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; ++i) bad += h1[i] != h2[i];
    printf("R=%d gpr-idx shared table vs per-slot chain: %s (%d mismatches)\n", R, bad ? "MISMATCH" : "identical", bad);
    delete[] h1; delete[] h2;
  }
  for (int wps : {2, 4, 8}) {
    const int blocks = cus * wps;
    const int iters = 4000;
    const double t0 = run<R, 0>(d, blocks, iters), t1 = run<R, 1>(d, blocks, iters),
                 t2 = run<R, 2>(d, blocks, iters);
    const double t3 = run3<R>(d, blocks, iters);
    const double n = wps * R;   // row dispatches per SIMD per iteration
    printf("R=%2d code=%3d KiB waves/SIMD=%d  straight %.2f  chain-random %.2f  chain-same %.2f  gidx-shared %.2f  ns per row per SIMD\n",
           R, R * 256 * BLKB / 1024, wps, t0 / n, t1 / n, t2 / n, t3 / n);
  }
}

int main()
{
  uint32_t* d;
  (void)hipMalloc(&d, 8192 * 256 * 4);
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  sweep<1>(d, cus);
  sweep<2>(d, cus);
  sweep<4>(d, cus);
  sweep<8>(d, cus);
  sweep<16>(d, cus);
  return 0;
}
'''


def main():
    src = SRC.replace("BLKB", str(BLK) + "u")
    b0 = ["if constexpr (R == %d) { %s }" % (R, straight(R)) for R in (1, 2, 4, 8, 16)]
    b1 = ["if constexpr (R == %d) { %s }" % (R, chain(R)) for R in (1, 2, 4, 8, 16)]
    b3 = ["if constexpr (R == %d) { %s }" % (R, gidx_chain(R)) for R in (1, 2, 4, 8, 16)]
    src = src.replace("BODY0", "\n      ".join(b0)).replace("BODY1", "\n      ".join(b1))
    src = src.replace("BODY3", "\n    ".join(b3))
    open(os.path.join(HERE, "microbench_fr.hip"), "w").write(src)


if __name__ == "__main__":
    main()
