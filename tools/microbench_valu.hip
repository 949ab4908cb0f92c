// VALU throughput microbenchmark for gfx950: independent chains of one instruction type.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(X) X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void kern(uint32_t* out, uint32_t seed, int iters)
{
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13,
           a6 = a0 * 17, a7 = a0 * 19;
  uint32_t s = seed * 0x9E3779B9u, t = seed + 12345;
  for (int i = 0; i < iters; ++i) {
#define STEP(x)                                                                                   \
    if constexpr (OP == 0) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(x) : "v"(s), "v"(t));   \
    else if constexpr (OP == 1) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(s), "v"(t)); \
    else if constexpr (OP == 2) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(s));            \
    else if constexpr (OP == 3) asm volatile("v_perm_b32 %0, %1, %2, %0" : "+v"(x) : "s"(s), "v"(t)); \
    else asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(s), "v"(t));
    REP8(STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7))
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
double run(uint32_t* d, int blocks, int iters)
{
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  kern<OP><<<blocks, 256>>>(d, 1, iters);
  hipEventRecord(e0);
  kern<OP><<<blocks, 256>>>(d, 1, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double wave_instr = double(blocks) * 4 * iters * 64;
  return wave_instr / (ms * 1e-3);
}

int main()
{
  uint32_t* d;
  hipMalloc(&d, 4096 * 256 * 4);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char* names[] = {"v_perm_b32 (vgpr)", "v_bitop3_b32", "v_xor_b32", "v_perm_b32 (sgpr src)", "v_and_or_b32"};
  for (int blocks : {cus * 2, cus * 4, cus * 8}) {
    double r[5] = {run<0>(d, blocks, 4096), run<1>(d, blocks, 4096), run<2>(d, blocks, 4096),
                   run<3>(d, blocks, 4096), run<4>(d, blocks, 4096)};
    for (int i = 0; i < 5; ++i)
      printf("blocks=%d %-24s %.3e wave-instr/s  = %.3f per SIMD per ns\n", blocks, names[i], r[i],
             r[i] / (cus * 4) / 1e9);
  }
  return 0;
}
