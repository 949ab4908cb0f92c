// CPU access speed of host memory the GPU can reach (per-packet adaptor design probe):
// malloc'd, hipHostMalloc'd (default / non-coherent / write-combined) and malloc + hipHostRegister,
// each written and read in 1 KiB pieces by the CPU the way the adaptor touches payloads, and
// read by a device kernel (one pass, PCIe).  usage: pinned_probe [MiB]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

// NUMA node of the page at p (move_pages with no target nodes only reports), -1 if unknown
static int page_node(void* p)
{
  void* pages[1] = {p};
  int status[1] = {-1};
  if (syscall(SYS_move_pages, 0, 1UL, pages, nullptr, status, 0) != 0) return -1;
  return status[0];
}

__global__ void sum_kernel(const uint4* p, size_t n, uint32_t* out)
{
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) *out = acc;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv)
{
  const size_t mib = argc > 1 ? atoi(argv[1]) : 64, n = mib << 20, piece = 1024;
  std::vector<uint8_t> src(n, 7), dst(n);
  uint32_t* dout;
  (void)hipMalloc(&dout, 4);
  struct K { const char* name; uint8_t* p; } ks[6];
  ks[0] = {"malloc", static_cast<uint8_t*>(aligned_alloc(4096, n))};
  (void)hipHostMalloc(&ks[1].p, n, hipHostMallocDefault); ks[1].name = "hipHostMalloc default";
  (void)hipHostMalloc(&ks[2].p, n, hipHostMallocNonCoherent); ks[2].name = "hipHostMalloc noncoherent";
  (void)hipHostMalloc(&ks[3].p, n, hipHostMallocWriteCombined); ks[3].name = "hipHostMalloc writecombined";
  ks[4] = {"malloc + hipHostRegister", static_cast<uint8_t*>(aligned_alloc(4096, n))};
  if (hipHostRegister(ks[4].p, n, hipHostRegisterMapped) != hipSuccess) printf("register failed\n");
  (void)hipHostMalloc(&ks[5].p, n, hipHostMallocNumaUser); ks[5].name = "hipHostMalloc numauser";
  int dev_numa = -1;
  (void)hipDeviceGetAttribute(&dev_numa, hipDeviceAttributeHostNumaId, 0);
  unsigned cpu = 0, node = 0;
  (void)syscall(SYS_getcpu, &cpu, &node, nullptr);
  printf("{\"cpu\": %u, \"cpu_numa\": %u, \"gpu_host_numa\": %d}\n", cpu, node, dev_numa);
  for (auto& k : ks) {
    memset(k.p, 1, n);
    double best_w = 1e9, best_r = 1e9, best_g = 1e9, best_rr = 1e9;
    for (int rep = 0; rep < 3; ++rep) {
      double t0 = now();
      for (size_t o = 0; o < n; o += piece) memcpy(k.p + o, src.data() + o, piece);   // CPU writes
      double t1 = now();
      for (size_t o = 0; o < n; o += piece) memcpy(dst.data() + o, k.p + o, piece);   // CPU reads
      double t2 = now();
      // 1 KiB pieces in a scattered order (the adaptor's access pattern: payloads of many flows)
      size_t o = 0;
      const size_t np = n / piece;
      for (size_t j = 0; j < np; ++j) {
        o = (o + 7919 * piece) % n;
        memcpy(dst.data() + o, k.p + o, piece);
      }
      double t3 = now();
      best_w = std::min(best_w, t1 - t0);
      best_r = std::min(best_r, t2 - t1);
      best_rr = std::min(best_rr, t3 - t2);
      void* dp = k.p;
      if (k.p != ks[0].p) {
        (void)hipHostGetDevicePointer(&dp, k.p, 0);
        hipEvent_t a, b;
        (void)hipEventCreate(&a); (void)hipEventCreate(&b);
        (void)hipEventRecord(a);
        hipLaunchKernelGGL(sum_kernel, dim3(1024), dim3(256), 0, 0, static_cast<const uint4*>(dp), n / 16, dout);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        best_g = std::min(best_g, ms * 1e-3);
      }
    }
    printf("{\"memory\": \"%s\", \"page_numa\": %d, \"cpu_write_GBps\": %.2f, \"cpu_read_GBps\": %.2f, "
           "\"cpu_scattered_read_GBps\": %.2f, \"gpu_read_GBps\": %.2f}\n",
           k.name, page_node(k.p), n / best_w / 1e9, n / best_r / 1e9, n / best_rr / 1e9,
           best_g < 1e8 ? n / best_g / 1e9 : 0.0);
  }
  return 0;
}
