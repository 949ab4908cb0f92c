// ntc_capi.cpp -- the reference's per-packet C ABI (netcode/c/*.h) on top of the MI355X engine.
//
// The protocol state machines (ntc::encoder, ntc::decoder, detail::decoder, packetizer) run on
// the host exactly as in the reference; every GF(2^8) region operation they issue -- a repair
// (detail/encoder.cc:15-64), the reduction of a repair by known sources (detail/decoder.cc:
// 393-408), peeling (:156-178) and full decoding (:480-559) -- is one ntc_gf256_combine_batch
// launch on the GPU.  There is no CPU fallback: without a HIP device ntc_new_encoder /
// ntc_new_decoder return NULL and ntc_* calls report an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "netcode/c/decoder.h"
#include "netcode/c/encoder.h"
#include "netcode/c/ext.h"
#include "netcode/gpu.h"
#include "gf256_field.hh"

namespace ntcx {

// ------------------------------------------------------------------------------ errors ----
struct packet_type_error : std::runtime_error {
  packet_type_error() : std::runtime_error("packet type error") {}
};
struct overflow_error : std::runtime_error {
  overflow_error() : std::runtime_error("overflow error") {}
};
struct device_error : std::runtime_error {
  explicit device_error(const std::string& m) : std::runtime_error(m) {}
};

// ------------------------------------------------------------- pinned payload blocks ----
// Every byte buffer of the adaptor (data objects, packets, payload nodes: `bytes` below) is a
// block of pinned host memory when a HIP device is present: the GPU then reads a new payload
// straight from the buffer the application filled (an upload job of the flush's first launch, one
// PCIe read) and writes each result straight into the buffer its node keeps -- no staging copy
// in, no copy out (DESIGN.md §3 batching).  The slabs are malloc'd pages pinned by
// hipHostRegister, so they sit on the NUMA node of the CPU thread that touches every byte:
// hipHostMalloc places them on the GPU's node, which on a box whose CPUs are on the other socket
// made CPU reads 25 % slower (tools/pinned_probe.hip); the GPU reads either over PCIe at the same
// rate.  Size classes: n rounded up to 1/8 of its power of
// two (64 B .. 128 KiB), carved from 4 MiB slabs that are never returned (the
// adaptor's peak payload memory stays reserved for the process); larger buffers, and every buffer
// without a device (or in the host-stub build), are malloc'd.  A spin lock guards the free lists.
class BlockPool {
 public:
  static BlockPool& get()
  {
    static BlockPool* p = new BlockPool;       // never destroyed (blocks outlive static teardown)
    return *p;
  }
  static constexpr size_t kMaxBlock = size_t(128) << 10;
  bool pinned() const { return pinned_; }
  // whether a buffer of capacity n came from the pinned pool
  bool pooled(size_t n) const { return pinned_ && n <= kMaxBlock; }
  void* alloc(size_t n)
  {
    if (!pooled(n)) {
      void* p = std::malloc(n ? n : 1);      // 16-byte aligned on x86-64 (alignof(max_align_t))
      if (!p) throw std::bad_alloc();
      return p;
    }
    const int c = cls(n);
    lock();
    void* p;
    if (!free_[c].empty()) {
      p = free_[c].back();
      free_[c].pop_back();
    } else {
      p = carve(csize(c));
      // room for every block of the class on its free list, so release() never allocates
      if (p && ++carved_[c] > free_[c].capacity()) {
        try {
          free_[c].reserve(2 * carved_[c]);
        } catch (...) {
          unlock();
          throw;
        }
      }
    }
    unlock();
    if (!p) throw std::bad_alloc();
    return p;
  }
  void release(void* p, size_t n)
  {
    if (!pooled(n)) {
      std::free(p);
      return;
    }
    const int c = cls(n);
    lock();
    free_[c].push_back(p);     // (the free lists live outside the blocks: taking a block touches
    unlock();                  // none of its cold bytes)
  }

 private:
  static constexpr size_t kSlab = size_t(4) << 20;
  static constexpr int kClasses = 12 * 8;      // 2^6 .. 2^17, 8 steps each
  BlockPool()
  {
#ifndef NTC_CAPI_HOST_STUB
    int n = 0;
    void* p = nullptr;
    // NTC_BATCH_PINNED_NUMA=gpu: slabs from hipHostMalloc, whose pages sit on the GPU's NUMA node
    // (A/B switch); default: malloc'd slabs pinned by hipHostRegister, so their pages are faulted
    // in on the NUMA node of the thread that first needs the pool -- the CPU side's node
    const char* numa = std::getenv("NTC_BATCH_PINNED_NUMA");
    gpu_node_ = numa && std::strcmp(numa, "gpu") == 0;
    if (std::getenv("NTC_BATCH_UNPINNED") == nullptr && hipGetDeviceCount(&n) == hipSuccess && n > 0 &&
        (p = new_slab()) != nullptr) {
      slab_ = static_cast<uint8_t*>(p);
      left_ = kSlab;
      pinned_ = true;
    } else {
      (void)hipGetLastError();
    }
#endif
  }
  // class of n: its power of two 2^k (k >= 6) in steps of 2^(k-3)
  static int cls(size_t n)
  {
    if (n <= 64) return 0;
    const int k = 64 - __builtin_clzll(n - 1);                // 2^(k-1) < n <= 2^k
    const size_t g = size_t(1) << (k - 3);
    const int j = static_cast<int>((n + g - 1) / g) - 4;       // 5..8 eighths -> 1..4 ... 
    return (k - 6) * 8 + (j < 0 ? 0 : j);
  }
  static size_t csize(int c)
  {
    const int k = c / 8 + 6, j = c % 8;
    return c == 0 ? 64 : (size_t(1) << (k - 3)) * static_cast<size_t>(j + 4);
  }
  void* carve(size_t b)                        // under the lock
  {
#ifndef NTC_CAPI_HOST_STUB
    if (left_ < b) {                           // a new slab (the old one's tail, < 128 KiB, stays unused)
      void* p = new_slab();
      if (!p) return nullptr;
      slab_ = static_cast<uint8_t*>(p);
      left_ = kSlab;
    }
#endif
    void* r = slab_;
    slab_ += b;
    left_ -= b;
    return r;
  }
#ifndef NTC_CAPI_HOST_STUB
  // a 4 MiB slab the device reads and writes through the same address as the host (on the CPU
  // thread's NUMA node unless gpu_node_; hipHostMalloc when registering is refused or maps the
  // pages at another device address)
  void* new_slab()
  {
    void* p = nullptr;
    if (!gpu_node_) {
      p = std::aligned_alloc(4096, kSlab);
      if (p && hipHostRegister(p, kSlab, hipHostRegisterMapped) == hipSuccess) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess && dp == p) return p;
        (void)hipHostUnregister(p);
      }
      (void)hipGetLastError();
      std::free(p);
      p = nullptr;
    }
    if (hipHostMalloc(&p, kSlab, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return p;
  }
#endif
  void lock() { while (lk_.test_and_set(std::memory_order_acquire)) {} }
  void unlock() { lk_.clear(std::memory_order_release); }
  std::atomic_flag lk_ = ATOMIC_FLAG_INIT;
  bool pinned_ = false;
  bool gpu_node_ = false;
  uint8_t* slab_ = nullptr;
  size_t left_ = 0;
  std::vector<void*> free_[kClasses];
  size_t carved_[kClasses] = {};
};

// --------------------------------------------------------------------- aligned storage ----
template <typename T>
struct Align16 {
  using value_type = T;
  Align16() = default;
  template <typename U> Align16(const Align16<U>&) {}
  // blocks of BlockPool: pinned when a device is present, else malloc's (16-byte aligned on
  // x86-64; glibc's memalign path, which the aligned operator new takes, bypasses its thread cache)
  T* allocate(size_t n) { return static_cast<T*>(BlockPool::get().alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) { BlockPool::get().release(p, n * sizeof(T)); }
  // resize(n) default-initialises (no zeroing), like the reference's byte_buffer (buffer.hh:66-73);
  // resize(n, 0) and assign(n, 0) still zero-fill
  template <typename U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <typename U, typename... A> void construct(U* p, A&&... a)
  {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
  template <typename U> bool operator==(const Align16<U>&) const { return true; }
  template <typename U> bool operator!=(const Align16<U>&) const { return false; }
};
using bytes = std::vector<uint8_t, Align16<uint8_t>>;

// ------------------------------------------------------------------ resident payloads ----
// The batching adaptor (class Batch below) keeps every payload it combines on the device: a
// payload is uploaded once, at the first flush that needs it, into a chunk of the device arena,
// and the results that later combinations read (decoded sources, reduced repairs) stay there too.
// A chunk is reused once no live payload points into it.
// NTC_BATCH_PROFILE=1: where a batch flush spends its host time (seconds, summed over flushes),
// printed to stderr at exit.  Diagnostics only; off by default (one getenv at load).
struct BatchProf {
  const bool on = std::getenv("NTC_BATCH_PROFILE") != nullptr;
  double complete = 0, emit_prev = 0, roots = 0, walk = 0, stage = 0, enqueue = 0, wait = 0, emit = 0;
  uint64_t flushes = 0, jobs = 0, terms = 0, up_bytes = 0, down_bytes = 0;
  static double now()
  {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  ~BatchProf()
  {
    if (on && flushes)
      std::fprintf(stderr,
                   "{\"batch_profile\": {\"flushes\": %llu, \"jobs\": %llu, \"terms\": %llu, \"up_bytes\": %llu, "
                   "\"down_bytes\": %llu, \"complete_s\": %.6f, \"emit_prev_s\": %.6f, \"roots_s\": %.6f, "
                   "\"walk_s\": %.6f, \"stage_s\": %.6f, \"enqueue_s\": %.6f, \"wait_s\": %.6f, \"emit_s\": %.6f}}\n",
                   (unsigned long long)flushes, (unsigned long long)jobs, (unsigned long long)terms,
                   (unsigned long long)up_bytes, (unsigned long long)down_bytes, complete, emit_prev, roots,
                   walk, stage, enqueue, wait, emit);
  }
};
static BatchProf g_prof;
#define NTC_PROF_T(var) const double var = g_prof.on ? BatchProf::now() : 0.0
#define NTC_PROF_ADD(field, since) do { if (g_prof.on) g_prof.field += BatchProf::now() - (since); } while (0)

struct DevChunk {
  uint8_t* d = nullptr;
  size_t cap = 0, used = 0;
  std::atomic<long> live{0};
};

// Small host objects of the adaptor (payload nodes with their shared-pointer control blocks,
// expression term arrays) from per-size free lists: a flush releases hundreds of them at once,
// more than glibc's per-thread cache keeps, and malloc's slower bins showed up as ≈ 10 % of the
// encoder's host time (sampling profile, DESIGN §3 batching).  64-byte classes up to 4 KiB, carved
// from 256 KiB malloc'd chunks that are never returned; a spin lock guards the lists.
class SmallPool {
 public:
  static SmallPool& get()
  {
    static SmallPool* p = new SmallPool;       // never destroyed (objects outlive static teardown)
    return *p;
  }
  static constexpr size_t kMax = 4096;
  void* alloc(size_t n)
  {
    if (n > kMax) return ::operator new(n);
    const size_t c = (n + 63) / 64;
    lock();
    void* p = free_[c];
    if (p) {
      free_[c] = *static_cast<void**>(p);
    } else {
      const size_t b = c * 64;
      if (left_ < b) {
        chunk_ = static_cast<uint8_t*>(std::malloc(kChunk));
        left_ = chunk_ ? kChunk : 0;
      }
      if (chunk_ && left_ >= b) {
        p = chunk_;
        chunk_ += b;
        left_ -= b;
      }
    }
    unlock();
    if (!p) throw std::bad_alloc();
    return p;
  }
  void release(void* p, size_t n) noexcept
  {
    if (n > kMax) {
      ::operator delete(p);
      return;
    }
    const size_t c = (n + 63) / 64;
    lock();
    *static_cast<void**>(p) = free_[c];
    free_[c] = p;
    unlock();
  }

 private:
  static constexpr size_t kChunk = size_t(256) << 10;
  void lock() { while (lk_.test_and_set(std::memory_order_acquire)) {} }
  void unlock() { lk_.clear(std::memory_order_release); }
  std::atomic_flag lk_ = ATOMIC_FLAG_INIT;
  uint8_t* chunk_ = nullptr;
  size_t left_ = 0;
  void* free_[kMax / 64 + 1] = {};
};

template <typename T>
struct SmallAlloc {
  using value_type = T;
  SmallAlloc() = default;
  template <typename U> SmallAlloc(const SmallAlloc<U>&) {}
  T* allocate(size_t n) { return static_cast<T*>(SmallPool::get().alloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) noexcept { SmallPool::get().release(p, n * sizeof(T)); }
  template <typename U> bool operator==(const SmallAlloc<U>&) const { return true; }
  template <typename U> bool operator!=(const SmallAlloc<U>&) const { return false; }
};

struct Node;
using NodeRef = std::shared_ptr<Node>;
constexpr uint32_t kNoPos = ~0u;
constexpr uint32_t kDirect = ~0u - 1;     // a root's result goes straight into its own pinned buffer
// c * (the first len bytes of node's payload, zero-extended).  hold keeps the input alive; it is
// empty when the expression's owner guarantees that instead (an encoder's repair terms: the
// encoder keeps every source a pending repair reads, Encoder::grave_) -- two atomic reference-
// count operations fewer per term, 32 per repair.
struct Term {
  Node* node;
  NodeRef hold;
  uint32_t c;
  uint16_t len;
  Term(NodeRef n, uint32_t c_, uint16_t len_) : node(n.get()), hold(std::move(n)), c(c_), len(len_) {}
  Term(Node* n, uint32_t c_, uint16_t len_) : node(n), c(c_), len(len_) {}
};
using Expr = std::vector<Term, SmallAlloc<Term>>;

// A payload: base (bytes handed in or received) or derived (a linear combination of other
// payloads, evaluated at a batch flush after everything it reads).  Immutable once created.
struct Node : std::enable_shared_from_this<Node> {
  bytes host;                  // base: the payload (from byte hoff on); derived: its value once fetched
  uint32_t hoff = 0;           // a received packet's buffer is adopted whole: payload offset in it
  uint16_t size = 0;
  uint32_t w = 8;              // field of a derived node's coefficients
  bool derived = false;
  bool done = false;           // derived: evaluated (on the device, or on the host for w != 8)
  bool fetched = false;        // derived: value in `host`
  Expr expr;                   // derived, until evaluated
  DevChunk* chunk = nullptr;   // device copy: chunk + byte offset (16-byte aligned, zero-padded)
  uint32_t off = 0;
  int level = 0;               // flush bookkeeping: evaluation level, visit stamp
  uint64_t mark = 0;
  uint32_t rpos = ~0u;         // during a flush: offset of the fetched value in the result staging
  ~Node()
  {
    if (chunk) chunk->live.fetch_sub(1, std::memory_order_relaxed);
  }
  bool has_value() const { return !derived || fetched; }
  const uint8_t* data() const { return host.data() + hoff; }
};

inline NodeRef base_node(const uint8_t* p, size_t n)
{
  auto nd = std::allocate_shared<Node>(SmallAlloc<Node>());
  nd->host.assign(p, p + n);
  nd->size = static_cast<uint16_t>(n);
  return nd;
}

// A base payload that takes over the buffer it lies in (a received packet): no copy.
inline NodeRef adopt_node(bytes&& buf, size_t off, size_t n)
{
  auto nd = std::allocate_shared<Node>(SmallAlloc<Node>());
  nd->host = std::move(buf);
  nd->hoff = static_cast<uint32_t>(off);
  nd->size = static_cast<uint16_t>(n);
  return nd;
}

inline NodeRef derived_node(uint32_t w, uint16_t size, Expr&& e)
{
  auto nd = std::allocate_shared<Node>(SmallAlloc<Node>());
  nd->derived = true;
  nd->w = w;
  nd->size = size;
  nd->expr = std::move(e);
  return nd;
}

// ---------------------------------------------------------------------- device engine ----
// One engine + stream + staging per process.  Encoders and decoders are not thread-safe (like the
// reference), but distinct objects may live on distinct threads (tests/end_to_end_mt.cc runs an
// encoder and a decoder on two threads), so every use of the shared staging holds mu_.
class Device {
 public:
  static Device& get()
  {
    // never destroyed: payload nodes may outlive static destruction order at process exit
    static Device* d = new Device;
    if (!d->eng_) throw device_error(d->err_);
    return *d;
  }

  // out[0..out_len) = sum_i c_i * in_i[0..len_i)  (inputs zero padded), one launch.
  void combine(uint32_t w, size_t n, const uint8_t* const* in, const uint16_t* lens,
               const uint32_t* coefs, size_t out_len, uint8_t* out)
  {
    uint8_t* outs[1] = {out};
    combine_rows(w, n ? n : 0, in, lens, 1, coefs, out_len, outs);
  }

  // Several outputs from the same inputs: out_s = sum_i coef[i][s] * in_i (full decoding).
  // GF(2^8): ntc_gf256_combine_batch (u8 coefficients, tile pitch); other fields:
  // ntc_gf_combine_batch (u32 coefficients).
  void combine_rows(uint32_t w, size_t n, const uint8_t* const* in, const uint16_t* lens,
                    size_t rows, const uint32_t* coef /*[n][rows]*/, size_t out_len,
                    uint8_t* const* out)
  {
    std::lock_guard<std::mutex> lock(mu_);
    size_t mx = out_len;
    for (size_t i = 0; i < n; ++i) mx = std::max<size_t>(mx, lens[i]);
    const size_t stride = std::max<size_t>(16, (mx + 15) / 16 * 16);
    const size_t nin = n ? n : 1;                  // an empty window combines a zero input
    const uint32_t pitch = w == 8 ? ntc_gf256_coef_pitch(static_cast<uint32_t>(rows))
                                  : static_cast<uint32_t>(4 * rows);
    grow(nin * stride, nin * pitch, rows * stride);
    std::memset(h_in_, 0, nin * stride);
    std::memset(h_coef_, 0, nin * pitch);
    for (size_t i = 0; i < n; ++i) {
      std::memcpy(h_in_ + i * stride, in[i], lens[i]);
      for (size_t s = 0; s < rows; ++s) {
        if (w == 8) h_coef_[i * pitch + s] = static_cast<uint8_t>(coef[i * rows + s]);
        else std::memcpy(h_coef_ + i * pitch + 4 * s, &coef[i * rows + s], 4);
      }
    }
#ifdef NTC_CAPI_HOST_STUB
    std::memset(h_out_, 0, rows * stride);
#else
    check(hipMemcpyAsync(d_in_, h_in_, nin * stride, hipMemcpyHostToDevice, stream_), "H2D");
    check(hipMemcpyAsync(d_coef_, h_coef_, nin * pitch, hipMemcpyHostToDevice, stream_), "H2D");
    const int rc = w == 8
        ? ntc_gf256_combine_batch(eng_, 1, static_cast<uint32_t>(nin), static_cast<uint32_t>(rows),
                                  static_cast<uint32_t>(stride), d_in_, d_coef_, d_out_, stream_)
        : ntc_gf_combine_batch(eng_, w, 1, static_cast<uint32_t>(nin), static_cast<uint32_t>(rows),
                               static_cast<uint32_t>(stride), d_in_,
                               reinterpret_cast<const uint32_t*>(d_coef_), d_out_, stream_);
    if (rc) throw device_error(ntc_gf256_last_error());
    check(hipMemcpyAsync(h_out_, d_out_, rows * stride, hipMemcpyDeviceToHost, stream_), "D2H");
    check(hipStreamSynchronize(stream_), "sync");
#endif
    for (size_t s = 0; s < rows; ++s) std::memcpy(out[s], h_out_ + s * stride, out_len);
  }

  // G independent combinations of up to k inputs each (batched repairs):
  //   out_g = sum_i c_gi * in_gi, inputs from fill(g, i, &ptr, &len, &c) (false past the last),
  //   each output handed to sink(g, bytes) -- one H2D, one launch, one D2H.
  template <typename Fill, typename Sink>
  void combine_generations(uint32_t w, size_t G, size_t k, size_t stride, Fill fill, Sink sink)
  {
    std::lock_guard<std::mutex> lock(mu_);
    combine_generations_locked(w, G, k, stride, fill, sink);
  }

  template <typename Fill, typename Sink>
  void combine_generations_body(uint32_t w, size_t G, size_t k, size_t stride, Fill fill, Sink sink)
  {
    const uint32_t pitch = w == 8 ? ntc_gf256_coef_pitch(1) : 4u;
    grow(G * k * stride, G * k * pitch, G * stride);
    std::memset(h_coef_, 0, G * k * pitch);
    for (size_t g = 0; g < G; ++g)
      for (size_t i = 0; i < k; ++i) {
        uint8_t* dst = h_in_ + (g * k + i) * stride;
        const uint8_t* ptr = nullptr;
        uint16_t len = 0;
        uint32_t c = 0;
        if (!fill(g, i, &ptr, &len, &c)) { std::memset(dst, 0, stride); continue; }
        std::memcpy(dst, ptr, len);
        std::memset(dst + len, 0, stride - len);
        if (w == 8) h_coef_[(g * k + i) * pitch] = static_cast<uint8_t>(c);
        else std::memcpy(h_coef_ + (g * k + i) * pitch, &c, 4);
      }
#ifdef NTC_CAPI_HOST_STUB
    std::memset(h_out_, 0, G * stride);
#else
    check(hipMemcpyAsync(d_in_, h_in_, G * k * stride, hipMemcpyHostToDevice, stream_), "H2D");
    check(hipMemcpyAsync(d_coef_, h_coef_, G * k * pitch, hipMemcpyHostToDevice, stream_), "H2D");
    const int rc = w == 8
        ? ntc_gf256_combine_batch(eng_, static_cast<uint32_t>(G), static_cast<uint32_t>(k), 1,
                                  static_cast<uint32_t>(stride), d_in_, d_coef_, d_out_, stream_)
        : ntc_gf_combine_batch(eng_, w, static_cast<uint32_t>(G), static_cast<uint32_t>(k), 1,
                               static_cast<uint32_t>(stride), d_in_,
                               reinterpret_cast<const uint32_t*>(d_coef_), d_out_, stream_);
    if (rc) throw device_error(ntc_gf256_last_error());
    check(hipMemcpyAsync(h_out_, d_out_, G * stride, hipMemcpyDeviceToHost, stream_), "D2H");
    check(hipStreamSynchronize(stream_), "sync");
#endif
    for (size_t g = 0; g < G; ++g) sink(g, h_out_ + g * stride);
  }

  uint64_t launches() const { return launches_; }

  // Batch flush: evaluate every derived node the roots need (each after the nodes it reads),
  // then bring the roots' values to the host.  GF(2^8): payloads on the device arena, one
  // gather_combine launch per dependency level; other fields: per level one host-staged combine.
  // async (ntc_batch_set_async): enqueue the GF(2^8) work and return its flight id (0: nothing
  // left in flight); its results land in the nodes at complete_through(id) (other fields' work,
  // host-staged, completes here).  Two staging sets: a flush may be launched while the previous
  // one is still in flight; a third waits for the oldest.
  uint64_t evaluate(const std::vector<Node*>& roots, bool async = false)
  {
    std::lock_guard<std::mutex> lock(mu_);
    NTC_PROF_T(t_walk);
    const uint64_t ep = ++epoch_;
    std::vector<Node*> todo;                       // dependencies first
    std::vector<std::pair<Node*, size_t>> stack;
    for (Node* r : roots) {
      if (!r->derived || r->done || r->mark == ep) continue;
      r->mark = ep;
      stack.push_back({r, 0});
      while (!stack.empty()) {
        Node* n = stack.back().first;
        size_t& i = stack.back().second;
        if (i < n->expr.size()) {
          Node* c = n->expr[i++].node;
          if (c->derived && !c->done && c->mark != ep) {
            c->mark = ep;
            stack.push_back({c, 0});
          }
          continue;
        }
        int lv = 1;
        for (const Term& t : n->expr)
          if (t.node->derived && !t.node->done) lv = std::max(lv, t.node->level + 1);
        n->level = lv;
        todo.push_back(n);
        stack.pop_back();
      }
    }
    auto by_level = [](const Node* a, const Node* b) { return a->level < b->level; };
    if (!std::is_sorted(todo.begin(), todo.end(), by_level))   // (often one level: encoder repairs)
      std::stable_sort(todo.begin(), todo.end(), by_level);
    std::vector<Node*> t8, tw;
    for (Node* n : todo) (n->w == 8 ? t8 : tw).push_back(n);
    NTC_PROF_ADD(walk, t_walk);
    if (!tw.empty()) evaluate_host(tw);
    if (t8.empty() && roots.empty()) return 0;
    return evaluate_w8(t8, roots, ep, async);
  }

  // flights up to id complete: their work done, their roots' values in the nodes
  void complete_through(uint64_t id)
  {
    std::lock_guard<std::mutex> lock(mu_);
    while (!flights_.empty() && flights_.front().id <= id) complete_oldest_locked();
  }

  // every flight complete (device work done, roots' values in their nodes)
  void quiesce()
  {
    std::lock_guard<std::mutex> lock(mu_);
    while (!flights_.empty()) complete_oldest_locked();
  }

  // true when flight id's work is done (never waits)
  bool ready(uint64_t id)
  {
    std::lock_guard<std::mutex> lock(mu_);
    for (const Flight& f : flights_)
      if (f.id == id) {
#ifndef NTC_CAPI_HOST_STUB
        return hipEventQuery(st_[f.set].ev) == hipSuccess;
#else
        return true;
#endif
      }
    return true;                         // completed already
  }


 private:
  // w != 8: level by level, inputs from the host (the old per-field path)
  void evaluate_host(const std::vector<Node*>& todo)
  {
    for (size_t a = 0; a < todo.size();) {
      size_t b = a;
      while (b < todo.size() && todo[b]->level == todo[a]->level && todo[b]->w == todo[a]->w) ++b;
      size_t kmax = 1, mx = 16;
      for (size_t i = a; i < b; ++i) {
        kmax = std::max(kmax, todo[i]->expr.size());
        mx = std::max<size_t>(mx, todo[i]->size);
      }
      combine_generations_locked(todo[a]->w, b - a, kmax, (mx + 15) / 16 * 16,
          [&](size_t g, size_t i, const uint8_t** ptr, uint16_t* len, uint32_t* c) {
            const Node* n = todo[a + g];
            if (i >= n->expr.size()) return false;
            *ptr = n->expr[i].node->data();
            *len = n->expr[i].len;
            *c = n->expr[i].c;
            return true;
          },
          [&](size_t g, const uint8_t* sym) {
            Node* n = todo[a + g];
            n->host.assign(sym, sym + n->size);
            n->fetched = n->done = true;
            n->expr.clear();
          });
      a = b;
    }
  }

  static size_t pad16(size_t n) { return (std::max<size_t>(n, 1) + 15) / 16 * 16; }

  // a region of `need` bytes in the device arena (bump allocation in the current chunk; a chunk
  // no live payload points into is reused, else a new one is added)
  DevChunk* arena_alloc(size_t need, size_t* off)
  {
    if (!cur_ || cur_->cap - cur_->used < need) {
      cur_ = nullptr;
      for (DevChunk* c : chunks_)
        if (c->cap >= need && c->live.load(std::memory_order_relaxed) == 0) { cur_ = c; c->used = 0; break; }
      if (!cur_) {
        auto* c = new DevChunk;
        c->cap = std::max<size_t>(need, size_t(16) << 20);
#ifdef NTC_CAPI_HOST_STUB
        c->d = static_cast<uint8_t*>(std::malloc(c->cap));
#else
        check(hipMalloc(&c->d, c->cap), "hipMalloc arena");
#endif
        chunks_.push_back(c);
        cur_ = c;
      }
    }
    *off = cur_->used;
    cur_->used += need;
    return cur_;
  }

  // One flush of GF(2^8) jobs: the payloads the jobs read that are not on the device yet and the
  // job / term descriptors go up in ONE copy into the flush's arena region; a root's result is
  // written by its job both into the arena and straight into pinned host memory (the job's second
  // output), so a flush is one copy, one launch per dependency level and one synchronisation.
  uint64_t evaluate_w8(const std::vector<Node*>& todo, const std::vector<Node*>& roots, uint64_t ep,
                       bool async)
  {
    NTC_PROF_T(t_stage);
    const uint64_t up_mark = ep + (1ull << 63);
    // new payloads: in pinned blocks the device pulls them itself (upload jobs), others are
    // staged into the flush's copy
    BlockPool& pool = BlockPool::get();
    std::vector<Node*> up, pull;
    size_t up_bytes = 0, pull_bytes = 0, out_bytes = 0, nterms = 0;
    uint32_t pull_max = 1;
    for (Node* n : todo) {
      nterms += n->expr.size();
      out_bytes += pad16(n->size);
      for (const Term& t : n->expr) {
        Node* c = t.node;
        if (c->chunk || (c->derived && !c->done) || c->mark == up_mark) continue;
        c->mark = up_mark;
        if (pool.pooled(c->host.capacity()) && c->size) {
          pull.push_back(c);
          pull_bytes += pad16(c->size);
          pull_max = std::max<uint32_t>(pull_max, c->size);
        } else {
          up.push_back(c);
          up_bytes += pad16(c->size);
        }
      }
    }
    // results the host needs: roots evaluated now (second output: straight into the node's own
    // pinned buffer, or the staging set's results) and earlier (device copy)
    size_t root_bytes = 0, late_bytes = 0;
    std::vector<Node*> late;
    for (Node* r : roots) {
      if (!r->derived || r->fetched) continue;
      const bool direct = pool.pinned();
      if (direct) r->host.resize(r->size);         // a pooled block (sizes <= 65535)
      if (!r->done) {
        if (direct) {
          r->rpos = kDirect;
        } else {
          r->rpos = static_cast<uint32_t>(root_bytes);
          root_bytes += pad16(r->size);
        }
      } else if (r->chunk) {
        late.push_back(r);
        if (!direct) late_bytes += pad16(r->size);
      }
    }
    if (todo.empty() && late.empty()) return 0;
    // a staging set with no flight in it (else wait for the oldest flight)
    int si = !st_[0].busy ? 0 : !st_[1].busy ? 1 : -1;
    if (si < 0) {
      // a busy set always has its flight queued (complete_oldest_locked); checked all the same
      if (flights_.empty()) throw device_error("batch staging sets busy with no flight queued");
      si = flights_.front().set;
      complete_oldest_locked();
    }
    Stage& S = st_[si];
    // flush region of the arena: [staged payloads | descriptors | pulled payloads | job outputs];
    // descriptors: the upload jobs (one term each) first, then the combination jobs
    const size_t npull = pull.size(), njobs = npull + todo.size();
    const size_t desc = pad16(njobs * sizeof(ntc_gf256_gather_job) + (npull + nterms) * sizeof(ntc_gf256_gather_term));
    const size_t region = up_bytes + (todo.empty() ? 0 : desc) + pull_bytes + out_bytes;
    size_t base = 0;
    DevChunk* ch = region ? arena_alloc(region, &base) : nullptr;
    grow_stage(S, up_bytes + desc, root_bytes + late_bytes);
    uint8_t* const h_up = S.up;
    uint8_t* const h_down = S.down;
    size_t pos = 0;
    for (Node* c : up) {
      std::memcpy(h_up + pos, c->data(), c->size);
      std::memset(h_up + pos + c->size, 0, pad16(c->size) - c->size);
      c->chunk = ch;
      c->off = static_cast<uint32_t>(base + pos);
      ch->live.fetch_add(1, std::memory_order_relaxed);
      pos += pad16(c->size);
    }
    auto* jobs = reinterpret_cast<ntc_gf256_gather_job*>(h_up + up_bytes);
    auto* terms = reinterpret_cast<ntc_gf256_gather_term*>(h_up + up_bytes + njobs * sizeof(ntc_gf256_gather_job));
    size_t ti = 0, opos = base + up_bytes + desc;
    for (size_t j = 0; j < npull; ++j) {           // upload jobs: 1 * the payload, read over PCIe once
      Node* c = pull[j];
      c->chunk = ch;
      c->off = static_cast<uint32_t>(opos);
      ch->live.fetch_add(1, std::memory_order_relaxed);
      opos += pad16(c->size);
      jobs[j] = ntc_gf256_gather_job{reinterpret_cast<uint64_t>(ch->d + c->off), 0, static_cast<uint32_t>(ti), 1,
                                     c->size, 0};
      terms[ti++] = ntc_gf256_gather_term{reinterpret_cast<uint64_t>(c->data()), c->size, 1};
    }
    for (size_t j = 0; j < todo.size(); ++j) {
      Node* n = todo[j];
      n->chunk = ch;
      n->off = static_cast<uint32_t>(opos);
      ch->live.fetch_add(1, std::memory_order_relaxed);
      opos += pad16(n->size);
      const uint64_t out2 = n->rpos == kDirect ? reinterpret_cast<uint64_t>(n->host.data())
                          : n->rpos != kNoPos ? reinterpret_cast<uint64_t>(h_down + n->rpos) : 0;
      jobs[npull + j] = ntc_gf256_gather_job{reinterpret_cast<uint64_t>(ch->d + n->off), out2,
                                             static_cast<uint32_t>(ti), static_cast<uint32_t>(n->expr.size()),
                                             n->size, 0};
      for (const Term& t : n->expr)
        terms[ti++] = ntc_gf256_gather_term{reinterpret_cast<uint64_t>(t.node->chunk->d + t.node->off),
                                            std::min<uint32_t>(t.len, n->size), t.c};
    }
    NTC_PROF_ADD(stage, t_stage);
    if (g_prof.on) {
      g_prof.jobs += todo.size();
      g_prof.terms += nterms;
      g_prof.up_bytes += up_bytes + desc;
      g_prof.down_bytes += root_bytes + late_bytes;
    }
#ifndef NTC_CAPI_HOST_STUB
    NTC_PROF_T(t_enq);
    if (!todo.empty())
      check(hipMemcpyAsync(ch->d + base, h_up, up_bytes + desc, hipMemcpyHostToDevice, stream_), "H2D payloads + jobs");
    const auto* djobs = reinterpret_cast<const ntc_gf256_gather_job*>(todo.empty() ? nullptr : ch->d + base + up_bytes);
    const auto* dterms = reinterpret_cast<const ntc_gf256_gather_term*>(
        todo.empty() ? nullptr : ch->d + base + up_bytes + njobs * sizeof(ntc_gf256_gather_job));
    if (npull && ntc_gf256_gather_combine(eng_, static_cast<uint32_t>(npull), djobs, dterms, pull_max, stream_))
      throw device_error(ntc_gf256_last_error());
    for (size_t a = 0; a < todo.size();) {
      size_t b = a;
      uint32_t m = 1;
      while (b < todo.size() && todo[b]->level == todo[a]->level) m = std::max<uint32_t>(m, todo[b++]->size);
      if (ntc_gf256_gather_combine(eng_, static_cast<uint32_t>(b - a), djobs + npull + a, dterms, m, stream_))
        throw device_error(ntc_gf256_last_error());
      a = b;
    }
    size_t lp = root_bytes;
    for (Node* r : late) {
      if (pool.pinned()) {                       // straight into the node's pinned buffer
        r->rpos = kDirect;
        if (r->size)
          check(hipMemcpyAsync(r->host.data(), r->chunk->d + r->off, r->size, hipMemcpyDeviceToHost, stream_), "D2H");
        continue;
      }
      r->rpos = static_cast<uint32_t>(lp);
      check(hipMemcpyAsync(h_down + lp, r->chunk->d + r->off, pad16(r->size), hipMemcpyDeviceToHost, stream_), "D2H");
      lp += pad16(r->size);
    }
    check(hipEventRecord(S.ev, stream_), "hipEventRecord");
    NTC_PROF_ADD(enqueue, t_enq);
#else
    std::memset(h_down, 0, root_bytes + late_bytes);
    size_t lp = root_bytes;
    for (Node* r : late) {
      r->rpos = static_cast<uint32_t>(lp);
      lp += pad16(r->size);
    }
#endif
    ++launches_;
    // the flight: the nodes count as resident for later launches (stream order); the record
    // keeps every node alive (an expression's terms hold its inputs' arena chunks) and remembers
    // where each root's value lands in the set's results
    Flight f;
    f.id = next_flight_++;
    f.set = si;
    S.busy = true;
    for (Node* n : todo) {
      n->done = true;
      f.todo.push_back(n->shared_from_this());
    }
    for (Node* r : roots)
      if (r->derived && !r->fetched && r->rpos != kNoPos) {
        f.roots.emplace_back(r->shared_from_this(), r->rpos);
        r->rpos = kNoPos;
      }
    flights_.push_back(std::move(f));
    if (async) return flights_.back().id;
    // synchronous: this flight and any older one
    while (!flights_.empty()) complete_oldest_locked();
    return 0;
  }

  // flushes launched and not yet completed, oldest first, each in its own staging set
  struct Stage {
    uint8_t *up = nullptr, *down = nullptr;      // pinned: uploads + descriptors / results
    size_t cap_up = 0, cap_down = 0;
    hipEvent_t ev = nullptr;                     // recorded after the set's last copy
    bool busy = false;                           // a flight in it
  };
  struct Flight {
    uint64_t id = 0;
    int set = 0;
    std::vector<NodeRef> todo;
    std::vector<std::pair<NodeRef, uint32_t>> roots;   // root, offset of its value in set.down
  };
  Stage st_[2];
  std::deque<Flight> flights_;
  uint64_t next_flight_ = 1;

  void wait_event(hipEvent_t ev)
  {
#ifndef NTC_CAPI_HOST_STUB
    // poll ~50 us (a flush's usual device time), then block: a long flush does not burn a core
    hipError_t e;
    const auto t0 = std::chrono::steady_clock::now();
    while ((e = hipEventQuery(ev)) == hipErrorNotReady)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50)) {
        e = hipEventSynchronize(ev);
        break;
      }
    check(e, "hipEventQuery");
#else
    (void)ev;
#endif
  }

  // the oldest flight: wait for its work, then its roots' values into the nodes (a copy out of
  // pinned memory: reading the pinned results in place at every use measured slower)
  // If the wait fails (it throws), the flight stays queued and its staging set stays busy: the
  // queue and the sets never disagree, and a later call waits for the same flight again.
  void complete_oldest_locked()
  {
    NTC_PROF_T(t_c);
    Stage& S = st_[flights_.front().set];
    {
      NTC_PROF_T(t_wait);
      wait_event(S.ev);
      NTC_PROF_ADD(wait, t_wait);
    }
    Flight f = std::move(flights_.front());
    flights_.pop_front();
    S.busy = false;
    for (const NodeRef& n : f.todo) n->expr.clear();
    for (auto& rp : f.roots) {
      Node* r = rp.first.get();
      if (r->fetched) continue;
      if (rp.second != kDirect) r->host.assign(S.down + rp.second, S.down + rp.second + r->size);
      r->hoff = 0;                               // (kDirect: the job wrote the node's own buffer)
      r->fetched = true;
    }
    NTC_PROF_ADD(complete, t_c);
  }

  void grow_stage(Stage& S, size_t up, size_t down)
  {
    auto up_h = [](uint8_t** h, size_t* cap, size_t need) {
      if (need <= *cap) return;
      const size_t n = std::max(need, *cap * 2);
#ifdef NTC_CAPI_HOST_STUB
      std::free(*h);
      *h = static_cast<uint8_t*>(std::malloc(n));
#else
      if (*h) (void)hipHostFree(*h);
      *h = nullptr;
      check(hipHostMalloc(reinterpret_cast<void**>(h), n, hipHostMallocDefault), "hipHostMalloc");
#endif
      *cap = n;
    };
    up_h(&S.up, &S.cap_up, up + 16);
    up_h(&S.down, &S.cap_down, down + 16);
  }

  // combine_generations without taking mu_ (the caller holds it)
  template <typename Fill, typename Sink>
  void combine_generations_locked(uint32_t w, size_t G, size_t k, size_t stride, Fill fill, Sink sink);

  Device()
  {
#ifdef NTC_CAPI_HOST_STUB
    eng_ = reinterpret_cast<ntc_gf256_engine*>(this);
    return;
#endif
    const char* v = std::getenv("NTC_DEVICE");
    const int dev = v ? std::atoi(v) : 0;
    if (ntc_gf256_engine_create(dev, &eng_) != 0) {
      err_ = std::string("no MI355X engine: ") + ntc_gf256_last_error();
      eng_ = nullptr;
      return;
    }
    if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
      err_ = "hipStreamCreate failed";
      ntc_gf256_engine_destroy(eng_);
      eng_ = nullptr;
      return;
    }
    if (hipEventCreateWithFlags(&st_[0].ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&st_[1].ev, hipEventDisableTiming) != hipSuccess) {
      err_ = "hipEventCreate failed";
      ntc_gf256_engine_destroy(eng_);
      eng_ = nullptr;
      return;
    }
    try {
      warm_up();
    } catch (const std::exception& e) {
      err_ = e.what();
      ntc_gf256_engine_destroy(eng_);
      eng_ = nullptr;
    }
  }

  // Once per process, when the first encoder / decoder is made: pinned staging and a first
  // arena chunk, and one flush-shaped round trip (copy engine, gather kernel) so that no
  // first-use initialisation (tens of ms on a fresh process) lands in a packet's call.
  void warm_up()
  {
    grow_stage(st_[1], size_t(4) << 20, size_t(4) << 20);
    grow_stage(st_[0], size_t(4) << 20, size_t(4) << 20);
    uint8_t* const h_up_ = st_[0].up;
    uint8_t* const h_down_ = st_[0].down;
    size_t off = 0;
    DevChunk* ch = arena_alloc(96, &off);        // [source 16 | job 32 | term 16 | output 16]
    auto* job = reinterpret_cast<ntc_gf256_gather_job*>(h_up_ + 16);
    auto* term = reinterpret_cast<ntc_gf256_gather_term*>(h_up_ + 16 + sizeof(ntc_gf256_gather_job));
    std::memset(h_up_, 0, 16);
    *term = ntc_gf256_gather_term{reinterpret_cast<uint64_t>(ch->d + off), 16, 1};
    *job = ntc_gf256_gather_job{reinterpret_cast<uint64_t>(ch->d + off + 64), reinterpret_cast<uint64_t>(h_down_),
                                0, 1, 16, 0};
    check(hipMemcpyAsync(ch->d + off, h_up_, 64, hipMemcpyHostToDevice, stream_), "warm-up H2D");
    // a flush-sized copy too: large copies take another path (copy engine) with its own first use
    size_t boff = 0;
    DevChunk* bch = arena_alloc(size_t(512) << 10, &boff);
    check(hipMemcpyAsync(bch->d + boff, h_up_, size_t(512) << 10, hipMemcpyHostToDevice, stream_), "warm-up H2D");
    if (ntc_gf256_gather_combine(eng_, 1, reinterpret_cast<const ntc_gf256_gather_job*>(ch->d + off + 16),
                                 reinterpret_cast<const ntc_gf256_gather_term*>(ch->d + off + 16 + sizeof(ntc_gf256_gather_job)),
                                 16, stream_))
      throw device_error(ntc_gf256_last_error());
    check(hipMemcpyAsync(h_down_ + 16, ch->d + off + 64, 16, hipMemcpyDeviceToHost, stream_), "warm-up D2H");
    check(hipStreamSynchronize(stream_), "warm-up sync");
    cur_->used = 0;                              // the chunk holds nothing live
  }
  ~Device()
  {
    // Process teardown: the HIP runtime may already be gone; release best effort.
  }
  static void check(hipError_t e, const char* what)
  {
    if (e != hipSuccess) throw device_error(std::string(what) + ": " + hipGetErrorString(e));
  }
  void grow(size_t in_bytes, size_t coef_bytes, size_t out_bytes)
  {
    auto up = [](void** d, void** h, size_t* cap, size_t need) {
      if (need <= *cap) return;
      const size_t n = std::max(need, *cap * 2);
      if (*d) (void)hipFree(*d);
      if (*h) (void)hipHostFree(*h);
      *d = nullptr;
      *h = nullptr;
      *cap = 0;
#ifdef NTC_CAPI_HOST_STUB
      *d = std::malloc(n);
      *h = std::malloc(n);
#else
      check(hipMalloc(d, n), "hipMalloc");
      check(hipHostMalloc(h, n, hipHostMallocDefault), "hipHostMalloc");
#endif
      *cap = n;
    };
    up(reinterpret_cast<void**>(&d_in_), reinterpret_cast<void**>(&h_in_), &cap_in_, in_bytes);
    up(reinterpret_cast<void**>(&d_coef_), reinterpret_cast<void**>(&h_coef_), &cap_coef_, coef_bytes + 64);
    up(reinterpret_cast<void**>(&d_out_), reinterpret_cast<void**>(&h_out_), &cap_out_, out_bytes);
    ++launches_;
  }

  std::mutex mu_;
  ntc_gf256_engine* eng_ = nullptr;
  hipStream_t stream_ = nullptr;
  std::string err_;
  uint8_t *d_in_ = nullptr, *h_in_ = nullptr, *d_coef_ = nullptr, *h_coef_ = nullptr;
  uint8_t *d_out_ = nullptr, *h_out_ = nullptr;
  size_t cap_in_ = 0, cap_coef_ = 0, cap_out_ = 0;
  uint64_t launches_ = 0;
  // resident payload arena and its staging (GF(2^8) batches)
  std::vector<DevChunk*> chunks_;
  DevChunk* cur_ = nullptr;
  uint64_t epoch_ = 0;
};

template <typename Fill, typename Sink>
void Device::combine_generations_locked(uint32_t w, size_t G, size_t k, size_t stride, Fill fill, Sink sink)
{
  combine_generations_body(w, G, k, stride, fill, sink);
}

// galois_field (galois_field.hh:18-167) for the field size an encoder / decoder was built with:
// GF(2^8) through the engine's tables, w in {4, 16, 32} through ntc_gf_* (gpu.h).
struct Field {
  uint32_t w;
  explicit Field(uint32_t w_) : w(w_)
  {
    if (w != 4 && w != 8 && w != 16 && w != 32)
      throw std::invalid_argument("galois field size must be 4, 8, 16 or 32");
  }
  // w = 8 inline (the engine library's compile-time tables): these run per window source of
  // every repair, so no call through the shared library's PLT
  uint32_t coef(uint32_t rid, uint32_t sid) const
  {
    return w == 8 ? ntcgpu::coefficient(rid, sid) : ntc_gf_coefficient(w, rid, sid);
  }
  uint16_t msize(uint16_t s, uint32_t c) const
  {
    if (w != 8) return ntc_gf_multiply_size(w, s, c);
    const uint8_t cc = static_cast<uint8_t>(c);       // galois_field.hh:108-115 (bytewise)
    return static_cast<uint16_t>(ntcgpu::field_mul(cc, static_cast<uint8_t>(s & 0xFF)) |
                                 (ntcgpu::field_mul(cc, static_cast<uint8_t>(s >> 8)) << 8));
  }
  uint32_t mul(uint32_t a, uint32_t b) const
  {
    return w == 8 ? ntc_gf256_multiply(static_cast<uint8_t>(a), static_cast<uint8_t>(b))
                  : ntc_gf_multiply(w, a, b);
  }
  uint32_t inv(uint32_t a) const
  {
    return w == 8 ? ntc_gf256_invert(static_cast<uint8_t>(a)) : ntc_gf_invert(w, a);
  }
};

// --------------------------------------------------------------------------- wire format ----
// Big-endian fields; id lists RLE-coded on 16-bit deltas (detail/packetizer.hh:263-352).
struct Writer {
  ntc_packet_handler h;
  bytes* buf = nullptr;        // set: packets are built into *buf instead of going to h
  void raw(const void* p, size_t n)
  {
    if (buf) buf->insert(buf->end(), static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + n);
    else h.prepare_packet(h.context, static_cast<const char*>(p), n);
  }
  void u8(uint8_t x) { raw(&x, 1); }
  void u16(uint16_t x) { const uint8_t b[2] = {uint8_t(x >> 8), uint8_t(x)}; raw(b, 2); }
  void u32(uint32_t x)
  {
    const uint8_t b[4] = {uint8_t(x >> 24), uint8_t(x >> 16), uint8_t(x >> 8), uint8_t(x)};
    raw(b, 4);
  }
  void ids(const std::vector<uint32_t>& v)      // packetizer.hh:263-309
  {
    if (v.empty()) { u16(0); return; }
    // runs of equal differences: counted first (the count leads), then written
    auto runs = [&v](auto&& emit) {
      size_t c = 1;
      while (c < v.size()) {
        uint8_t run = 1;
        const uint32_t d = v[c] - v[c - 1];
        while (c + 1 < v.size() && v[c + 1] - v[c] == d && run < 255) { ++run; ++c; }
        emit(run, static_cast<uint16_t>(d));
        ++c;
      }
    };
    size_t nr = 0;
    runs([&nr](uint8_t, uint16_t) { ++nr; });
    u16(static_cast<uint16_t>(nr + 1));
    u32(v[0]);
    runs([this](uint8_t run, uint16_t d) { u8(run); u16(d); });
  }
  void end() { if (!buf) h.send_packet(h.context); }
};

struct Reader {
  const uint8_t* p;
  size_t left;
  uint8_t u8() { need(1); const uint8_t x = p[0]; p += 1; left -= 1; return x; }
  uint16_t u16() { need(2); const uint16_t x = uint16_t((p[0] << 8) | p[1]); p += 2; left -= 2; return x; }
  uint32_t u32()
  {
    need(4);
    const uint32_t x = (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3];
    p += 4; left -= 4;
    return x;
  }
  const uint8_t* skip(size_t n) { need(n); const uint8_t* q = p; p += n; left -= n; return q; }
  void need(size_t n) const { if (left < n) throw overflow_error(); }
  std::vector<uint32_t> ids()                   // packetizer.hh:312-352 (sorted, unique)
  {
    std::vector<uint32_t> v;
    ids_into(v);
    return v;
  }
  void ids_into(std::vector<uint32_t>& v)        // the same into v (cleared; capacity reused)
  {
    v.clear();
    const uint16_t ne = u16();
    if (ne == 0) return;
    uint32_t acc = u32();
    v.reserve(32);
    v.push_back(acc);
    bool sorted = true;                         // the writer's RLE of ascending ids: already a set
    for (uint32_t i = 0; i + 1u < ne; ++i) {
      const uint8_t run = u8();
      const uint16_t d = u16();
      for (uint32_t j = 0; j < run; ++j) {
        acc += d;
        sorted = sorted && acc > v.back();
        v.push_back(acc);
      }
    }
    if (!sorted) {                              // a hand-made list: the reference's std::set order
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
    }
  }
};

}  // namespace ntcx

// ====================================================================== C ABI objects ======
struct ntc_data_t {
  ntcx::bytes v;
};

struct ntc_packet_t {
  static constexpr size_t shift = 9;   // 16 - 7-byte header (packet.hh:30-36)
  ntcx::bytes v;
  explicit ntc_packet_t(size_t n) : v(n + shift, 0) {}
  // a packet handed to an encoder / decoder is moved from (empty, size 0) until resized
  uint8_t* data()
  {
    static uint8_t none[16];
    return v.size() >= shift ? v.data() + shift : none;
  }
  size_t size() const { return v.size() >= shift ? v.size() - shift : 0; }
};

namespace ntcx {

// ============================================================================== encoder ====
class Batch;
class Decoder;

// One event queued in a Batch, emitted at flush in production order: a packet (encoder source,
// encoder repair whose two symbol copies are filled at flush, decoder ack) or a decoder data
// delivery (the bytes of `node`, truncated to `size`).
struct Pending {
  enum Kind { ENC_PACKET, DEC_PACKET, DEC_DATA };
  Kind kind = ENC_PACKET;
  class Encoder* enc = nullptr;
  class Decoder* dec = nullptr;
  bytes pkt;                           // wire bytes
  NodeRef node;                        // encoder repair / delivered data: the payload to emit
  uint16_t size = 0;                   // repair symbol size / data size
  size_t off1 = 0, off2 = 0;           // encoder repair: where the two symbol copies go in pkt
                                       // (not stored there: emitted from the node, handlers.h)
};

class Encoder {
 public:
  Encoder(uint8_t w, ntc_packet_handler h) : f_(w), out_{h} { Device::get(); }
  Encoder(Encoder&&) = default;
  ~Encoder();

  // encoder.hh:255-285.  Returns the buffer of the source that left the window when nothing
  // else holds it (empty otherwise): the caller's data object takes it, so a steady stream of
  // items reuses the window's buffers instead of allocating one per item.
  bytes add_data(bytes&& d)
  {
    bytes spare;
    if (queued_ == 0 && !grave_.empty()) grave_.clear();   // no repair of ours pending any more
    if (window_.size() == window_size_) {
      NodeRef old = std::move(window_.front().sym);
      window_.pop_front();
      if (queued_ != 0) grave_.push_back(std::move(old));  // a pending repair may read it
      else if (old.use_count() == 1 && old->hoff == 0) spare = std::move(old->host);
    }
    auto nd = std::allocate_shared<Node>(SmallAlloc<Node>());
    nd->size = static_cast<uint16_t>(d.size());
    nd->host = std::move(d);
    window_.push_back(Src{cur_sid_, std::move(nd)});
    const Src& s = window_.back();
    if (systematic_) {
      ++nb_sources_;
      ++nb_sent_packets_;
      Pending p;
      p.enc = this;
      // unbatched, or an eager batch with nothing of this encoder waiting: a source packet needs
      // no GPU result, so it goes out now (the encoder's own sequence is unchanged)
      const bool now = emit_now();
      if (now) out_.buf = nullptr;
      else begin(p, 7 + s.sym->size);
      // packetizer.hh:165-183: the 7-byte header in one piece, then the payload
      const uint8_t hdr[7] = {2, uint8_t(s.id >> 24), uint8_t(s.id >> 16), uint8_t(s.id >> 8), uint8_t(s.id),
                              uint8_t(s.sym->size >> 8), uint8_t(s.sym->size)};
      out_.raw(hdr, 7);
      out_.raw(s.sym->data(), s.sym->size);
      out_.end();
      if (!now) finish(std::move(p));
    } else {
      generate_repair();
    }
    if ((cur_sid_ + 1) % rate_ == 0) generate_repair();
    ++cur_sid_;
    return spare;
  }

  // encoder.hh:162-169, 321-333 + detail/encoder.cc:15-64 (the combination runs on the GPU; with
  // a Batch attached it is deferred to the batch's flush, one launch for every pending repair)
  void generate_repair()
  {
    if (window_.empty()) throw std::runtime_error("generate_repair on an empty window");
    ids_.clear();
    uint16_t symsz = 0, esz = 0;
    Expr terms;
    if (batch_) terms.reserve(window_.size());
    else { in_.clear(); lens_.clear(); cs_.clear(); }
    // encoded size = XOR of msize(len_i, c_i) (detail/encoder.cc:38, 61-62); with equal lengths
    // (the usual case) that is msize(len, XOR of c_i) -- the product distributes over XOR -- so
    // one product per repair instead of one per source (w = 8 and w = 4: bytewise size coding)
    const uint16_t sz0 = window_.front().sym->size;
    bool same = f_.w <= 8;
    uint32_t cx = 0;
    for (const Src& s : window_) {
      const uint32_t c = f_.coef(cur_rid_, s.id);
      const uint16_t sz = s.sym->size;
      if (batch_) {
        terms.push_back(Term{s.sym.get(), c, sz});   // unheld (grave_); distinct sources: no merging
      } else {
        in_.push_back(s.sym->data());
        lens_.push_back(sz);
        cs_.push_back(c);
      }
      ids_.push_back(s.id);
      symsz = std::max<uint16_t>(symsz, sz);
      if (same && sz == sz0) cx ^= c;
      else {
        if (same) {                                // first unequal length: the per-source form
          same = false;
          esz = f_.msize(sz0, cx);
        }
        esz = static_cast<uint16_t>(f_.msize(sz, c) ^ esz);
      }
    }
    if (same) esz = f_.msize(sz0, cx);
    bytes sym;
    if (!batch_) {
      sym.resize(symsz);
      Device::get().combine(f_.w, in_.size(), in_.data(), lens_.data(), cs_.data(), symsz, sym.data());
    }
    const uint32_t rid = cur_rid_++;
    ++nb_repairs_;
    ++nb_sent_packets_;
    Pending p;
    p.enc = this;
    begin(p, 15 + 4 + 3 * ids_.size());
    out_.u8(1);                                    // packetizer.hh:90-122
    out_.u32(rid);
    out_.u16(symsz);
    p.off1 = batch_ ? p.pkt.size() : 0;
    if (!batch_) out_.raw(sym.data(), symsz);                // batched: emitted at flush
    out_.ids(ids_);
    out_.u16(esz);
    out_.u16(symsz);
    p.off2 = batch_ ? p.pkt.size() : 0;
    if (!batch_) out_.raw(sym.data(), symsz);
    out_.end();
    if (batch_) {
      p.size = symsz;
      p.node = derived_node(f_.w, symsz, std::move(terms));
    }
    finish(std::move(p));
  }

  void set_batch(Batch* b);
  void drop_batch();                   // the batch is going away: its queued events are discarded
  Batch* batch() const { return batch_; }
  bool emit_now() const;               // an event needing no GF result goes out at once
  size_t queued_ = 0;                  // this encoder's events waiting in its batch
  const ntc_packet_handler& handler() const { return out_.h; }

  // encoder.hh:290-318 + packetizer.hh:64-88 + source_list.hh:34-60
  size_t add_packet(const uint8_t* p, size_t n)
  {
    if (n == 0) throw overflow_error();
    if (p[0] != 0) throw packet_type_error();
    ++nb_acks_;
    Reader r{p, n};
    r.u8();
    const uint16_t nbp = r.u16();
    const std::vector<uint32_t> ids = r.ids();
    if (adaptive_) {
      double loss = 0.0;
      if (nb_sent_packets_ > 0)
        loss = static_cast<double>(int(nb_sent_packets_) - int(nbp)) / static_cast<double>(nb_sent_packets_);
      rate_ = loss < 0.01 ? 50 : static_cast<size_t>(std::ceil((1.0 / loss) / 2.0));
    }
    nb_sent_packets_ = 0;
    auto it = window_.begin();
    size_t ii = 0;
    while (it != window_.end() && ii < ids.size()) {
      if (it->id == ids[ii]) {
        if (queued_ != 0) grave_.push_back(std::move(it->sym));   // a pending repair may read it
        it = window_.erase(it);
        ++ii;
      }
      else if (it->id > ids[ii]) ++ii;
      else ++it;
    }
    return n - r.left;
  }

  size_t window() const { return window_.size(); }
  void set_rate(size_t r) { if (r) rate_ = r; }
  void set_window_size(size_t s) { if (s) window_size_ = s; }
  void set_systematic(bool s) { systematic_ = s; }
  void set_adaptive(bool a) { adaptive_ = a; }
  size_t counter(int which) const
  {
    switch (which) {
      case NTC_ENC_NB_SENT_REPAIRS: return nb_repairs_;
      case NTC_ENC_NB_SENT_SOURCES: return nb_sources_;
      case NTC_ENC_NB_RECEIVED_ACKS: return nb_acks_;
      case NTC_ENC_RATE: return rate_;
      case NTC_ENC_WINDOW: return window_.size();
      default: return 0;
    }
  }

 private:
  struct Src {
    uint32_t id;
    NodeRef sym;                       // immutable once in the window (shared with pending repairs)
  };
  // batch mode: the packet is built into p.pkt (begin) and queued in the batch (finish)
  void begin(Pending& p, size_t reserve);
  void finish(Pending&& p);

  Field f_;
  Writer out_;
  Batch* batch_ = nullptr;
  std::deque<Src> window_;
  std::vector<uint32_t> ids_, cs_;     // scratch of generate_repair
  // sources that left the window while repairs of ours were queued (their terms do not hold
  // them): released once nothing of ours is queued -- every queued repair has been evaluated,
  // emitted and dropped by then
  std::vector<NodeRef> grave_;
  std::vector<const uint8_t*> in_;
  std::vector<uint16_t> lens_;
  size_t rate_ = 5;
  size_t window_size_ = static_cast<size_t>(-1);
  bool systematic_ = true;
  bool adaptive_ = false;
  uint32_t cur_sid_ = 0, cur_rid_ = 0;
  size_t nb_repairs_ = 0, nb_acks_ = 0, nb_sources_ = 0;
  uint16_t nb_sent_packets_ = 0;
};

// ------------------------------------------------------------------------ flow containers ----
// A decoder's state spans one window of ids (tens of entries), inserted mostly at the back and
// dropped from the front: sorted vectors, not node-based trees -- no allocation per packet once the
// window is warm, and the same ordered iteration as the reference's std::map / std::set.  An
// insert or erase invalidates iterators and references into the container (the Decoder re-finds
// by key after any structural change).
template <class K, class V>
class FlatMap {
 public:
  using value_type = std::pair<K, V>;
  using iterator = typename std::vector<value_type>::iterator;
  using const_iterator = typename std::vector<value_type>::const_iterator;
  iterator begin() { return v_.begin(); }
  iterator end() { return v_.end(); }
  const_iterator begin() const { return v_.begin(); }
  const_iterator end() const { return v_.end(); }
  size_t size() const { return v_.size(); }
  bool empty() const { return v_.empty(); }
  void clear() { v_.clear(); }
  iterator lower_bound(K k)
  {
    if (v_.empty() || v_.back().first < k) return v_.end();        // the common case: a new id
    return std::lower_bound(v_.begin(), v_.end(), k, [](const value_type& a, K b) { return a.first < b; });
  }
  iterator find(K k)
  {
    auto it = lower_bound(k);
    return it != v_.end() && it->first == k ? it : v_.end();
  }
  size_t count(K k) { return find(k) != v_.end(); }
  std::pair<iterator, bool> emplace(K k, V&& v)
  {
    auto it = lower_bound(k);
    if (it != v_.end() && it->first == k) return {it, false};
    return {v_.emplace(it, k, std::move(v)), true};
  }
  V& operator[](K k)
  {
    auto it = lower_bound(k);
    if (it == v_.end() || it->first != k) it = v_.emplace(it, k, V());
    return it->second;
  }
  iterator erase(iterator it) { return v_.erase(it); }
  iterator erase(iterator a, iterator b) { return v_.erase(a, b); }
  size_t erase(K k)
  {
    auto it = find(k);
    if (it == v_.end()) return 0;
    v_.erase(it);
    return 1;
  }

 private:
  std::vector<value_type> v_;
};

// The in-order decoder's ids held back behind a gap.
class OrderedIds {
 public:
  using iterator = std::vector<uint32_t>::iterator;
  iterator begin() { return v_.begin(); }
  iterator end() { return v_.end(); }
  bool empty() const { return v_.empty(); }
  iterator find(uint32_t x)
  {
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    return it != v_.end() && *it == x ? it : v_.end();
  }
  iterator erase(iterator it) { return v_.erase(it); }
  void insert(uint32_t x)
  {
    if (v_.empty() || v_.back() < x) { v_.push_back(x); return; }
    auto it = std::lower_bound(v_.begin(), v_.end(), x);
    if (*it != x) v_.insert(it, x);
  }

 private:
  std::vector<uint32_t> v_;
};

// A sorted set of ids; up to kInline of them without a heap block (a missing source is usually
// covered by one to three repairs).
class IdSet {
 public:
  static constexpr uint32_t kInline = 6;
  IdSet() = default;
  IdSet(const IdSet& o) : n_(o.n_), big_(o.big_) { std::copy(o.in_, o.in_ + kInline, in_); }
  IdSet(IdSet&& o) noexcept : n_(o.n_), big_(std::move(o.big_)) { std::copy(o.in_, o.in_ + kInline, in_); o.n_ = 0; }
  IdSet& operator=(IdSet&& o) noexcept
  {
    n_ = o.n_;
    big_ = std::move(o.big_);
    std::copy(o.in_, o.in_ + kInline, in_);
    o.n_ = 0;
    return *this;
  }
  const uint32_t* begin() const { return big_.empty() ? in_ : big_.data(); }
  const uint32_t* end() const { return begin() + n_; }
  size_t size() const { return n_; }
  bool empty() const { return n_ == 0; }
  void insert(uint32_t x)
  {
    const uint32_t* b = begin();
    const size_t i = static_cast<size_t>(std::lower_bound(b, b + n_, x) - b);
    if (i < n_ && b[i] == x) return;
    if (big_.empty() && n_ < kInline) {
      std::copy_backward(in_ + i, in_ + n_, in_ + n_ + 1);
      in_[i] = x;
    } else {
      if (big_.empty()) big_.assign(in_, in_ + n_);
      big_.insert(big_.begin() + static_cast<std::ptrdiff_t>(i), x);
    }
    ++n_;
  }
  void erase(uint32_t x)
  {
    uint32_t* b = big_.empty() ? in_ : big_.data();
    uint32_t* e = b + n_;
    uint32_t* it = std::lower_bound(b, e, x);
    if (it == e || *it != x) return;
    if (big_.empty()) std::copy(it + 1, e, it);
    else big_.erase(big_.begin() + (it - b));
    --n_;
  }

 private:
  uint32_t n_ = 0;
  uint32_t in_[kInline] = {};
  std::vector<uint32_t> big_;  // past kInline ids (then the ids live here)
};

// ============================================================================== decoder ====
// detail/decoder.{hh,cc} semantics; host containers, GPU region work.
class Decoder {
 public:
  Decoder(uint8_t w, bool in_order, ntc_packet_handler ph, ntc_data_handler dh)
      : f_(w), in_order_(in_order), out_{ph}, dh_(dh), last_ack_(std::chrono::steady_clock::now())
  {
    Device::get();
  }
  Decoder(Decoder&&) = default;
  ~Decoder();

  void set_batch(Batch* b);
  void drop_batch() { batch_ = nullptr; queued_ = 0; }
  const ntc_packet_handler& packet_handler() const { return out_.h; }
  size_t queued_ = 0;                  // this decoder's events waiting in its batch
  const ntc_data_handler& data_handler() const { return dh_; }

  // decoder.hh:88-122.  own: the buffer p lies in, when the caller hands it over (the C ABI
  // moves the packet in, like the reference): a batched decoder keeps the payload in it.
  size_t add_packet(const uint8_t* p, size_t n, bytes* own = nullptr)
  {
    if (n == 0) throw overflow_error();
    Reader rd{p, n};
    const uint8_t ty = rd.u8();
    if (ty == 1) {
      ++nb_rrep_;
      ++ack_packets_;
      const uint32_t id = rd.u32();
      const uint16_t symsz = rd.u16();
      const uint8_t* sym = rd.skip(symsz);
      rd.ids_into(ids_);                           // (scratch: no allocation per repair)
      const uint16_t esz = rd.u16();
      const size_t consumed = n - rd.left;
      if (!ids_.empty()) on_repair(id, ids_, esz, sym, symsz, own);
      return consumed;
    }
    if (ty == 2) {
      ++nb_rsrc_;
      ++ack_packets_;
      const uint32_t id = rd.u32();
      const uint16_t sz = rd.u16();
      const uint8_t* sym = rd.skip(sz);
      const size_t consumed = n - rd.left;
      on_source(id, sym, sz, own);
      return consumed;
    }
    throw packet_type_error();
  }

  // decoder.hh:213-228
  void generate_ack()
  {
    std::vector<uint32_t> ids;
    ids.reserve(sources_.size());
    for (const auto& kv : sources_) ids.push_back(kv.first);
    Pending p;
    p.kind = Pending::DEC_PACKET;
    p.dec = this;
    const bool now = emit_now();                   // unbatched, or eager with nothing waiting
    out_.buf = now ? nullptr : &p.pkt;
    out_.u8(0);
    out_.u16(ack_packets_);
    out_.ids(ids);
    out_.end();
    out_.buf = nullptr;
    if (!now) queue(std::move(p));
    ++nb_acks_;
    ack_packets_ = 0;
  }

  void set_ack_period(size_t ms) { ack_period_ms_ = ms; }
  void set_ack_nb_packets(uint16_t nb) { if (nb) ack_nb_packets_ = std::min<uint16_t>(nb, 128); }

  size_t counter(int which) const
  {
    switch (which) {
      case NTC_DEC_NB_DECODED: return nb_decoded_;
      case NTC_DEC_NB_FAILED_FULL_DECODINGS: return nb_failed_;
      case NTC_DEC_NB_MISSING_SOURCES: return missing_.size();
      case NTC_DEC_NB_RECEIVED_REPAIRS: return nb_rrep_;
      case NTC_DEC_NB_RECEIVED_SOURCES: return nb_rsrc_;
      case NTC_DEC_NB_SENT_ACKS: return nb_acks_;
      case NTC_DEC_NB_USELESS_REPAIRS: return nb_useless_;
      case NTC_DEC_NB_PENDING_REPAIRS: return repairs_.size();
      default: return 0;
    }
  }

 private:
  struct Src {
    uint32_t id;
    bytes sym;                   // immediate mode
    uint16_t size;
    NodeRef node;                // batch mode: the payload (received: base; decoded: derived)
  };
  struct Rep {
    uint32_t id;
    std::vector<uint32_t> ids;   // sorted
    uint16_t esz;
    bytes sym;                   // immediate mode
    uint16_t symsz;
    // batch mode: the reduced repair, its own payload first (held); the removed sources' terms do
    // not hold them -- every such source has an id >= first, and the decoder keeps the sources it
    // drops while a repair with a smaller or equal first id is alive (grave_)
    Expr red;
    uint32_t first = 0;          // the repair's first source id on the wire
  };
  // the terms of r.red, each holding its node (for an expression that outlives the repair)
  static Expr held(const Expr& red)
  {
    Expr e;
    e.reserve(red.size());
    for (const Term& t : red) e.push_back(Term{t.hold ? t.hold : t.node->shared_from_this(), t.c, t.len});
    return e;
  }

  void queue(Pending&& p);
 public:
  bool emit_now() const;
 private:
  // batch mode: the reduced repair as one payload (its own payload when nothing was removed)
  NodeRef repair_node(const Rep& r) const
  {
    if (r.red.size() == 1 && r.red[0].c == 1 && r.red[0].len >= r.symsz) return r.red[0].hold;
    return derived_node(f_.w, r.symsz, held(r.red));
  }
  // batch mode: c * (the reduced repair truncated to len), zero-extended to size bytes
  NodeRef scaled_repair(const Rep& r, uint32_t c, uint16_t len, uint16_t size) const
  {
    Expr e;
    e.reserve(r.red.size());
    for (const Term& t : r.red)
      e.push_back(Term{t.hold ? t.hold : t.node->shared_from_this(), f_.mul(t.c, c), std::min(t.len, len)});
    return derived_node(f_.w, size, std::move(e));
  }

  // decoder.hh:231-248, 292-300
  void deliver(const Src& s)
  {
    if (batch_ && emit_now() && s.node->has_value()) {
      // an eager batch, nothing of this decoder waiting, the bytes at hand (a received source)
      static const uint8_t zero[16] = {0};
      dh_.read_data(dh_.context, reinterpret_cast<const char*>(s.size ? s.node->data() : zero), s.size);
    } else if (batch_) {
      Pending p;                 // a decoded source's value, or anything behind a waiting event
      p.kind = Pending::DEC_DATA;
      p.dec = this;
      p.size = s.size;
      p.node = s.node;
      queue(std::move(p));
    } else {
      dh_.read_data(dh_.context, reinterpret_cast<const char*>(s.sym.data()), s.size);
    }
    maybe_ack();
  }

 public:
  // decoder.hh:231-248: ack once enough packets arrived or the ack period elapsed
  void maybe_ack()
  {
    if (ack_packets_ >= ack_nb_packets_) {
      generate_ack();
      last_ack_ = std::chrono::steady_clock::now();
    } else if (ack_period_ms_ != 0) {
      const auto now = std::chrono::steady_clock::now();
      if (now - last_ack_ >= std::chrono::milliseconds(ack_period_ms_)) {
        generate_ack();
        last_ack_ = now;
      }
    }
  }

 private:
  void deliver_id(uint32_t id)
  {
    auto it = sources_.find(id);
    if (it != sources_.end()) deliver(it->second);
  }

  // detail/decoder.cc:570-591
  void flush_ordered()
  {
    auto it = ordered_.find(first_missing_);
    if (it == ordered_.end()) return;
    for (;;) {
      deliver_id(*it);
      it = ordered_.erase(it);
      first_missing_ += 1;
      if (it == ordered_.end() || *it > first_missing_) break;
    }
  }

  // detail/decoder.cc:393-408 for several known sources at once (XOR order is irrelevant).
  void remove_sources_data(Rep& r, const std::vector<const Src*>& known)
  {
    if (known.empty()) return;
    if (batch_) {                // one term per source payload, whatever produced it
      r.red.reserve(r.red.size() + known.size());
      // encoded-size update: XOR of msize(size_i, c_i); equal sizes (the usual case) make that
      // one product of the XORed coefficients (galois_field.hh:96-120 is linear in c)
      const uint16_t sz0 = known.front()->size;
      bool same = f_.w <= 8;
      uint32_t cx = 0;
      for (const Src* s : known) {
        const uint32_t c = f_.coef(r.id, s->id);
        if (same && s->size == sz0) cx ^= c;
        else r.esz = static_cast<uint16_t>(f_.msize(s->size, c) ^ r.esz);
        r.red.push_back(Term{s->node.get(), c, std::min<uint16_t>(s->size, r.symsz)});   // unheld
      }
      if (cx) r.esz = static_cast<uint16_t>(f_.msize(sz0, cx) ^ r.esz);
      return;
    }
    std::vector<const uint8_t*> in{r.sym.data()};
    std::vector<uint16_t> lens{r.symsz};
    std::vector<uint32_t> cs{1};
    for (const Src* s : known) {
      const uint32_t c = f_.coef(r.id, s->id);
      r.esz = static_cast<uint16_t>(f_.msize(s->size, c) ^ r.esz);
      in.push_back(s->sym.data());
      lens.push_back(std::min<uint16_t>(s->size, r.symsz));
      cs.push_back(c);
    }
    Device::get().combine(f_.w, in.size(), in.data(), lens.data(), cs.data(), r.symsz, r.sym.data());
  }

  // detail/decoder.cc:156-178
  Src create_source_from_repair(const Rep& r)
  {
    const uint32_t sid = r.ids.front();
    const uint32_t inv = f_.inv(f_.coef(r.id, sid));
    const uint16_t sz = f_.msize(r.esz, inv);
    if (batch_) {
      Src s{sid, bytes(), sz, nullptr};
      s.node = scaled_repair(r, inv, std::min(sz, r.symsz), sz);
      nb_decoded_ += 1;
      return s;
    }
    Src s{sid, bytes(std::max<size_t>(sz, 1), 0), sz};
    const uint8_t* in = r.sym.data();
    const uint16_t len = std::min(sz, r.symsz);
    Device::get().combine(f_.w, 1, &in, &len, &inv, sz, s.sym.data());
    nb_decoded_ += 1;
    return s;
  }

  // detail/decoder.cc:33-50
  void on_source(uint32_t id, const uint8_t* sym, uint16_t sz, bytes* own = nullptr)
  {
    if (has_last_ && id < last_id_) return;
    if (sources_.count(id)) return;
    Src s{id, bytes(), sz, nullptr};
    if (batch_) s.node = own ? adopt_node(std::move(*own), sym - own->data(), sz) : base_node(sym, sz);
    else s.sym.assign(sym, sym + sz);
    if (!batch_ && s.sym.empty()) s.sym.resize(1, 0);
    add_source_recursive(std::move(s));
    attempt_full_decoding();
  }

  // detail/decoder.cc:54-152
  // ids: the repair's source ids (sorted; a scratch vector of the caller, read only)
  void on_repair(uint32_t id, const std::vector<uint32_t>& ids, uint16_t esz, const uint8_t* sym, uint16_t symsz,
                 bytes* own = nullptr)
  {
    if (has_last_ && ids.back() < last_id_) return;
    if (repairs_.count(id)) return;
    drop_outdated(ids.front());
    // known / missing split first (the reference walks the ids in reverse, decoder.cc:102-130;
    // the order only matters for XOR, which is order-free), so the stored repair is built once
    // with its remaining ids -- no id vector per repair beyond the one it keeps
    known_.clear();
    size_t nrem = 0;
    for (uint32_t sid : ids) {
      auto s = sources_.find(sid);
      if (s != sources_.end()) known_.push_back(&s->second);
      else ++nrem;
    }
    if (nrem == 0) { ++nb_useless_; return; }
    std::vector<uint32_t> remaining;
    remaining.reserve(nrem);
    for (uint32_t sid : ids)
      if (!sources_.count(sid)) {
        missing_[sid].insert(id);
        remaining.push_back(sid);
      }
    Rep& r = repairs_.emplace(id, Rep{id, std::move(remaining), esz, bytes(), symsz, {}, ids.front()}).first->second;
    if (batch_) {
      r.red.reserve(1 + known_.size());
      r.red.push_back(Term{own ? adopt_node(std::move(*own), sym - own->data(), symsz) : base_node(sym, symsz),
                           1, symsz});
    } else {
      r.sym.assign(sym, sym + symsz);
    }
    if (!batch_ && r.sym.empty()) r.sym.resize(1, 0);
    remove_sources_data(r, known_);
    if (r.ids.size() == 1) {
      Src s = create_source_from_repair(r);
      missing_.erase(s.id);
      repairs_.erase(id);
      add_source_recursive(std::move(s));
      return;
    }
    attempt_full_decoding();
  }

  // detail/decoder.cc:249-337
  void add_source_recursive(Src&& src)
  {
    if (!in_order_) {
      deliver(src);
    } else if (src.id == first_missing_) {
      deliver(src);
      first_missing_ += 1;
      flush_ordered();
    }
    auto m = missing_.find(src.id);
    if (m != missing_.end()) {
      const IdSet rids = m->second;
      for (uint32_t rid : rids) {
        auto r = repairs_.find(rid);
        if (r == repairs_.end()) continue;
        remove_sources_data(r->second, {&src});
        auto& v = r->second.ids;
        v.erase(std::find(v.begin(), v.end(), src.id));
      }
      missing_.erase(src.id);
    }
    for (auto mit = missing_.begin(); mit != missing_.end();) {
      if (mit->second.size() == 1) {
        auto r = repairs_.find(*mit->second.begin());
        if (r != repairs_.end() && r->second.ids.size() == 1) {
          Src dec = create_source_from_repair(r->second);
          const uint32_t cur = mit->first;
          repairs_.erase(r);
          missing_.erase(mit);
          add_source_recursive(std::move(dec));
          mit = missing_.lower_bound(cur);
          continue;
        }
      }
      ++mit;
    }
    const uint32_t sid = src.id;
    sources_.emplace(sid, std::move(src));
    if (in_order_ && sid > first_missing_) ordered_.insert(sid);
  }

  // detail/decoder.cc:341-389
  void drop_outdated(uint32_t id)
  {
    has_last_ = true;
    last_id_ = id;
    for (auto it = repairs_.begin(); it != repairs_.end();) {
      if (id > it->second.ids.front()) {
        for (uint32_t sid : it->second.ids) {
          auto m = missing_.find(sid);
          if (m != missing_.end()) m->second.erase(it->first);
        }
        it = repairs_.erase(it);
      } else {
        ++it;
      }
    }
    if (in_order_) {
      while (!ordered_.empty() && *ordered_.begin() < id) {
        deliver_id(*ordered_.begin());
        ordered_.erase(ordered_.begin());
      }
      if (first_missing_ < id) first_missing_ = id;
      flush_ordered();
    }
    // sources leaving: those a live repair's unheld terms may read (id >= its first id) wait in
    // grave_ until no such repair is left
    const auto cut = sources_.lower_bound(id);
    uint32_t keep_from = ~0u;                      // smallest first id of a live repair
    for (const auto& kv : repairs_) keep_from = std::min(keep_from, kv.second.first);
    if (batch_)
      for (auto it = sources_.begin(); it != cut; ++it)
        if (it->first >= keep_from && it->second.node) grave_.push_back({it->first, std::move(it->second.node)});
    sources_.erase(sources_.begin(), cut);
    missing_.erase(missing_.begin(), missing_.lower_bound(id));
    prune_grave(keep_from);
  }
  void prune_grave(uint32_t keep_from)
  {
    if (grave_.empty()) return;
    grave_.erase(std::remove_if(grave_.begin(), grave_.end(),
                                [keep_from](const std::pair<uint32_t, NodeRef>& g) { return g.first < keep_from; }),
                 grave_.end());
  }
  void prune_grave()
  {
    uint32_t keep_from = ~0u;
    for (const auto& kv : repairs_) keep_from = std::min(keep_from, kv.second.first);
    prune_grave(keep_from);
  }

  // detail/invert_matrix.cc:9-128 semantics: returns false on a singular matrix (the reference
  // then reports index rows-1); inv is the unique inverse otherwise.  M is [n][n] row-major,
  // row = repair, column = missing source (the reference's storage rows).
  bool invert(std::vector<uint32_t> M, size_t n, std::vector<uint32_t>& inv) const
  {
    inv.assign(n * n, 0);
    for (size_t i = 0; i < n; ++i) inv[i * n + i] = 1;
    for (size_t i = 0; i < n; ++i) {
      size_t p = i;
      while (p < n && M[p * n + i] == 0) ++p;
      if (p == n) return false;
      if (p != i)
        for (size_t k = 0; k < n; ++k) { std::swap(M[i * n + k], M[p * n + k]); std::swap(inv[i * n + k], inv[p * n + k]); }
      const uint32_t piv = f_.inv(M[i * n + i]);
      for (size_t k = 0; k < n; ++k) { M[i * n + k] = f_.mul(M[i * n + k], piv); inv[i * n + k] = f_.mul(inv[i * n + k], piv); }
      for (size_t j = 0; j < n; ++j) {
        if (j == i || M[j * n + i] == 0) continue;
        const uint32_t f = M[j * n + i];
        for (size_t k = 0; k < n; ++k) { M[j * n + k] ^= f_.mul(f, M[i * n + k]); inv[j * n + k] ^= f_.mul(f, inv[i * n + k]); }
      }
    }
    return true;
  }

  // detail/decoder.cc:536-559: store a fully decoded source and deliver it (in order or not)
  void insert_decoded(Src&& src)
  {
    const uint32_t sid = src.id;
    sources_.emplace(sid, std::move(src));
    if (!in_order_) {
      deliver_id(sid);
    } else if (sid == first_missing_) {
      deliver_id(sid);
      first_missing_ += 1;
      flush_ordered();
    } else {
      ordered_.insert(sid);
    }
  }

  // detail/decoder.cc:412-566
  void attempt_full_decoding()
  {
    if (repairs_.empty() || missing_.empty()) return;
    if (missing_.size() > repairs_.size()) return;
    const size_t n = repairs_.size();
    std::vector<const Rep*> reps;
    for (const auto& kv : repairs_) reps.push_back(&kv.second);
    std::vector<uint32_t> mids;
    for (const auto& kv : missing_) mids.push_back(kv.first);
    std::vector<uint32_t> M(n * n, 0), inv;
    for (size_t q = 0; q < n; ++q)
      for (size_t s = 0; s < n; ++s)
        if (std::binary_search(reps[q]->ids.begin(), reps[q]->ids.end(), mids[s]))
          M[q * n + s] = f_.coef(reps[q]->id, mids[s]);
    if (!invert(M, n, inv)) {                      // :448-468 drop the repair at index rows-1
      ++nb_failed_;
      auto last = std::prev(repairs_.end());
      for (uint32_t sid : last->second.ids) missing_[sid].erase(last->first);
      repairs_.erase(last);
      return;
    }
    // X = M^-1 R: x_s = sum_q inv[s][q] r_q ; sizes from the reduced encoded sizes (:484-497)
    std::vector<uint16_t> sizes(n, 0);
    for (size_t s = 0; s < n; ++s)
      for (size_t q = 0; q < n; ++q) {
        const uint32_t c = inv[s * n + q];
        if (c) sizes[s] = static_cast<uint16_t>(f_.msize(reps[q]->esz, c) ^ sizes[s]);
      }
    if (batch_) {                      // derived payloads, evaluated at the batch's flush
      std::vector<NodeRef> rn(n);
      for (size_t q = 0; q < n; ++q) rn[q] = repair_node(*reps[q]);
      for (size_t s = 0; s < n; ++s) {
        Expr e;
        for (size_t q = 0; q < n; ++q) {
          const uint32_t c = inv[s * n + q];
          const uint16_t len = std::min(sizes[s], reps[q]->symsz);
          if (c && len) e.push_back(Term{rn[q], c, len});
        }
        Src src{mids[s], bytes(1, 0), sizes[s], derived_node(f_.w, sizes[s], std::move(e))};
        insert_decoded(std::move(src));
      }
      nb_decoded_ += n;
      repairs_.clear();
      missing_.clear();
      return;
    }
    std::vector<Src> dec(n);
    std::vector<uint8_t*> outs(n);
    uint16_t mx = 0;
    for (size_t s = 0; s < n; ++s) {
      dec[s] = Src{mids[s], bytes(std::max<size_t>(sizes[s], 1), 0), sizes[s]};
      outs[s] = dec[s].sym.data();
      mx = std::max(mx, sizes[s]);
    }
    std::vector<const uint8_t*> in(n);
    std::vector<uint16_t> lens(n);
    std::vector<uint32_t> cf(n * n);
    for (size_t q = 0; q < n; ++q) {
      in[q] = reps[q]->sym.data();
      lens[q] = reps[q]->symsz;
      for (size_t s = 0; s < n; ++s) cf[q * n + s] = inv[s * n + q];
    }
    // one launch for all missing sources; bytes past each decoded size are dropped below
    std::vector<bytes> full(n, bytes(std::max<size_t>(mx, 1), 0));
    std::vector<uint8_t*> fo(n);
    for (size_t s = 0; s < n; ++s) fo[s] = full[s].data();
    Device::get().combine_rows(f_.w, n, in.data(), lens.data(), n, cf.data(), mx, fo.data());
    for (size_t s = 0; s < n; ++s) {
      // the reference reads min(src_sz, repair.symbol_size()) bytes of each repair (:523, :531)
      std::memcpy(dec[s].sym.data(), full[s].data(), sizes[s]);
      insert_decoded(std::move(dec[s]));
    }
    nb_decoded_ += n;
    repairs_.clear();
    missing_.clear();
  }

  Field f_;
  Batch* batch_ = nullptr;
  bool in_order_;
  Writer out_;
  ntc_data_handler dh_;
  std::vector<uint32_t> ids_;          // scratch of add_packet / on_repair
  std::vector<const Src*> known_;
  std::vector<std::pair<uint32_t, NodeRef>> grave_;   // dropped sources live repairs may read
  uint32_t first_missing_ = 0;
  OrderedIds ordered_;
  FlatMap<uint32_t, Src> sources_;
  FlatMap<uint32_t, Rep> repairs_;
  FlatMap<uint32_t, IdSet> missing_;
  bool has_last_ = false;
  uint32_t last_id_ = 0;
  size_t nb_useless_ = 0, nb_failed_ = 0, nb_decoded_ = 0;
  size_t nb_rrep_ = 0, nb_rsrc_ = 0, nb_acks_ = 0;
  uint16_t ack_packets_ = 0;
  uint16_t ack_nb_packets_ = 50;
  size_t ack_period_ms_ = 100;
  std::chrono::steady_clock::time_point last_ack_;
};

// ============================================================================ batching ====
// an online batching adaptor behind the per-packet encoder and decoder.
// Objects attached to a Batch queue every packet and data delivery they produce, in production
// order; their protocol state advances immediately (the reference's control flow never reads
// payload bytes), while every GF region result is kept as an expression over the payloads it came
// from.  flush() evaluates all pending expressions -- encoder repairs and decoder deliveries --
// with one combine launch per field size instead of one launch and one PCIe round trip per region
// operation, then emits the queue in order.  Each object's callback sequence is exactly the
// unbatched one; only the time of the callbacks moves to the flush.
class Batch {
 public:
  ~Batch();
  void attach(Encoder* e) { encs_.push_back(e); }
  void attach(Decoder* d) { decs_.push_back(d); }
  void detach(Encoder* e)
  {
    e->queued_ = 0;
    encs_.erase(std::remove(encs_.begin(), encs_.end(), e), encs_.end());
    q_.erase(std::remove_if(q_.begin(), q_.end(), [e](const Pending& p) { return p.enc == e; }),
             q_.end());
    for (InFlight& f : flights_)
      f.q.erase(std::remove_if(f.q.begin(), f.q.end(), [e](const Pending& p) { return p.enc == e; }), f.q.end());
  }
  void detach(Decoder* d)
  {
    d->queued_ = 0;
    decs_.erase(std::remove(decs_.begin(), decs_.end(), d), decs_.end());
    q_.erase(std::remove_if(q_.begin(), q_.end(), [d](const Pending& p) { return p.dec == d; }),
             q_.end());
    for (InFlight& f : flights_)
      f.q.erase(std::remove_if(f.q.begin(), f.q.end(), [d](const Pending& p) { return p.dec == d; }), f.q.end());
  }
  void push(Pending&& p) { q_.push_back(std::move(p)); }
  // a packet buffer of an already flushed event (empty, capacity kept), or a new one
  bytes take_buffer()
  {
    if (pool_.empty()) return bytes();
    bytes b = std::move(pool_.back());
    pool_.pop_back();
    b.clear();
    return b;
  }
  size_t pending() const
  {
    size_t n = q_.size();
    for (const InFlight& f : flights_) n += f.q.size();
    return n;
  }
  void flush();
  void drain()                           // every queued and in-flight event delivered
  {
    const bool a = async;
    async = false;
    flush();
    async = a;
  }
  // Asynchronous flushes (opt-in, ntc_batch_set_async): flush() delivers the events of earlier
  // flushes whose device work is done (in order, never waiting, except for a third flush while
  // two are in flight), then starts the device work of the queued ones and returns; they are
  // delivered by a later flush (flush until pending() is 0 to drain).  The device work of one
  // flush overlaps whatever the caller does until it is done.
  bool async = false;
  // Eager emission (opt-in, ntc_batch_set_eager): an event that needs no GF result -- a source
  // packet, a received source's delivery, an ack -- of an object with nothing queued goes out at
  // once instead of at the flush.
  bool eager = false;

 private:
  std::vector<Encoder*> encs_;
  std::vector<Decoder*> decs_;
  std::vector<Pending> q_;
  struct InFlight {                // an asynchronous flush's events, awaiting its device work
    uint64_t id;                   // Device flight (0: none of its own, waits behind the others)
    std::vector<Pending> q;
  };
  std::deque<InFlight> flights_;

  std::vector<Pending> spare_;   // the last flushed queue's storage, reused by the next one
  void emit(std::vector<Pending>& q);
  std::vector<bytes> pool_;      // flushed packets' buffers (no malloc / free per packet)
};

bool Encoder::emit_now() const { return !batch_ || (batch_->eager && queued_ == 0); }
bool Decoder::emit_now() const { return !batch_ || (batch_->eager && queued_ == 0); }

void Encoder::drop_batch()
{
  batch_ = nullptr;
  queued_ = 0;
  if (!grave_.empty()) {                // discarded repairs may still be on the device
    Device::get().quiesce();
    grave_.clear();
  }
}

Encoder::~Encoder()
{
  if (batch_) batch_->detach(this);
  // repairs of ours still in the device's flights read the graveyard's payloads (their uploads):
  // let that work finish before the buffers go back to the pool
  if (!grave_.empty()) Device::get().quiesce();
}

void Encoder::set_batch(Batch* b)
{
  if (b == batch_) return;
  if (batch_) {
    batch_->drain();                    // keep this encoder's packet order across the switch
    batch_->detach(this);
  }
  batch_ = b;
  if (b) b->attach(this);
}

void Encoder::begin(Pending& p, size_t reserve)
{
  out_.buf = batch_ ? &p.pkt : nullptr;
  if (batch_) {
    p.pkt = batch_->take_buffer();
    p.pkt.reserve(reserve);
  }
}

void Encoder::finish(Pending&& p)
{
  out_.buf = nullptr;
  if (batch_) {
    batch_->push(std::move(p));
    ++queued_;
  }
}

Decoder::~Decoder()
{
  if (batch_) batch_->detach(this);
}

void Decoder::set_batch(Batch* b)
{
  if (b == batch_) return;
  if (batch_) {
    batch_->drain();
    batch_->detach(this);
  }
  if (!b) {
    // back to immediate mode: the payloads the protocol state still holds become host bytes
    std::vector<NodeRef> rn;
    std::vector<Node*> roots;
    for (auto& kv : sources_)
      if (kv.second.node) roots.push_back(kv.second.node.get());
    for (auto& kv : repairs_) {
      rn.push_back(repair_node(kv.second));
      roots.push_back(rn.back().get());
    }
    if (!roots.empty()) Device::get().evaluate(roots);
    auto host_bytes = [](const Node& n, uint16_t size) {
      bytes v(n.data(), n.data() + std::min<size_t>(n.host.size() - n.hoff, size));
      v.resize(std::max<size_t>(size, 1), 0);
      return v;
    };
    for (auto& kv : sources_)
      if (kv.second.node) {
        kv.second.sym = host_bytes(*kv.second.node, kv.second.size);
        kv.second.node.reset();
      }
    size_t i = 0;
    for (auto& kv : repairs_) {
      kv.second.sym = host_bytes(*rn[i++], kv.second.symsz);
      kv.second.red.clear();
    }
  } else {
    // into batch mode: the held symbols become base payloads
    for (auto& kv : sources_)
      if (!kv.second.node) kv.second.node = base_node(kv.second.sym.data(), kv.second.size);
    for (auto& kv : repairs_)
      if (kv.second.red.empty())
        kv.second.red.push_back(Term{base_node(kv.second.sym.data(), kv.second.symsz), 1, kv.second.symsz});
  }
  batch_ = b;
  if (b) b->attach(this);
}

void Decoder::queue(Pending&& p)
{
  if (batch_) {
    batch_->push(std::move(p));
    ++queued_;
  }
}

Batch::~Batch()
{
  for (Encoder* e : encs_) e->drop_batch();      // pending events are discarded
  for (Decoder* d : decs_) d->drop_batch();
}

void Batch::flush()
{
  if (g_prof.on) ++g_prof.flushes;
  // earlier asynchronous flushes, oldest first (their events precede the queued ones): those
  // whose device work is done -- all of them when not asynchronous
  while (!flights_.empty()) {
    InFlight& f = flights_.front();
    if (async && f.id && !Device::get().ready(f.id)) break;
    if (f.id) Device::get().complete_through(f.id);
    NTC_PROF_T(t_ep);
    std::vector<Pending> q = std::move(f.q);
    flights_.pop_front();
    emit(q);
    NTC_PROF_ADD(emit_prev, t_ep);
  }
  // every payload the queued events emit: evaluated (with what it reads) and fetched, all fields
  // and objects of the batch together
  NTC_PROF_T(t_r);
  std::vector<Node*> roots;
  for (const Pending& p : q_)
    if (p.node && !p.node->has_value()) roots.push_back(p.node.get());
  NTC_PROF_ADD(roots, t_r);
  if (async) {
    const uint64_t id = roots.empty() ? 0 : Device::get().evaluate(roots, true);
    if (id || !flights_.empty()) {       // in flight, or behind flights not yet delivered
      if (!q_.empty()) flights_.push_back(InFlight{id, std::move(q_)});
      q_ = std::vector<Pending>();
      if (q_.capacity() < spare_.capacity()) q_.swap(spare_);
      return;
    }
  } else if (!roots.empty()) {
    Device::get().evaluate(roots);
  }
  NTC_PROF_T(t_e);
  std::vector<Pending> q;
  q.swap(q_);
  if (q_.capacity() < spare_.capacity()) q_.swap(spare_);   // keep the queue's storage warm
  emit(q);
  NTC_PROF_ADD(emit, t_e);
}

// the handlers of a flushed queue, in production order
void Batch::emit(std::vector<Pending>& q)
{
  for (Pending& p : q) {
    --(p.kind == Pending::ENC_PACKET ? p.enc->queued_ : p.dec->queued_);   // before its callback
    if (p.kind == Pending::DEC_DATA) {
      const ntc_data_handler& h = p.dec->data_handler();
      static const uint8_t zero[16] = {0};
      const uint8_t* d = p.size ? p.node->data() : zero;
      h.read_data(h.context, reinterpret_cast<const char*>(d), p.size);
      continue;
    }
    const ntc_packet_handler& h = p.kind == Pending::ENC_PACKET ? p.enc->handler()
                                                                : p.dec->packet_handler();
    const char* pk = reinterpret_cast<const char*>(p.pkt.data());
    if (p.node) {
      // encoder repair: the packet's pieces around the two copies of the symbol, the symbol
      // straight from its payload (prepare_packet may be called several times per packet,
      // handlers.h; packetizer.hh:90-122 writes a repair the same way)
      const char* sym = reinterpret_cast<const char*>(p.node->data());
      h.prepare_packet(h.context, pk, p.off1);
      h.prepare_packet(h.context, sym, p.size);
      h.prepare_packet(h.context, pk + p.off1, p.off2 - p.off1);
      h.prepare_packet(h.context, sym, p.size);
      if (p.pkt.size() > p.off2) h.prepare_packet(h.context, pk + p.off2, p.pkt.size() - p.off2);
    } else {
      h.prepare_packet(h.context, pk, p.pkt.size());
    }
    h.send_packet(h.context);
  }
  for (Pending& p : q)
    if (p.pkt.capacity() && pool_.size() < 16384) pool_.push_back(std::move(p.pkt));
  q.clear();
  if (q.capacity() > spare_.capacity()) spare_.swap(q);
}

// c/detail/check_error.hh: exceptions -> ntc_error (message in thread-local storage).
thread_local std::string t_msg;

template <typename Fn>
auto guarded(Fn&& fn, ntc_error* error) noexcept -> decltype(fn())
{
  error->type = ntc_no_error;
  try {
    return fn();
  } catch (const packet_type_error&) {
    error->type = ntc_packet_type_error;
  } catch (const overflow_error&) {
    error->type = ntc_overflow_error;
  } catch (const std::bad_alloc&) {
    error->type = ntc_no_memory;
  } catch (const std::exception& e) {
    error->type = ntc_unknown_error;
    t_msg = e.what();
    error->message = &t_msg[0];
  } catch (...) {
    error->type = ntc_unknown_error;
    t_msg = "unknown error";
    error->message = &t_msg[0];
  }
  return decltype(fn())();
}

}  // namespace ntcx

struct ntc_encoder_t {
  ntcx::Encoder e;
};
struct ntc_batch_t {
  ntcx::Batch b;
};
struct ntc_decoder_t {
  ntcx::Decoder d;
};

extern "C" {

// ----------------------------------------------------------------------------- data ----
ntc_data_t* ntc_new_data(uint16_t size) noexcept
{
  auto* d = new (std::nothrow) ntc_data_t;
  if (!d) return nullptr;
  try { d->v.assign(size, 0); } catch (...) { delete d; return nullptr; }
  return d;
}
ntc_data_t* ntc_new_data_from(const char* src, uint16_t size) noexcept
{
  auto* d = ntc_new_data(size);
  if (d && size) std::memcpy(d->v.data(), src, size);
  return d;
}
void ntc_delete_data(ntc_data_t* d) noexcept { delete d; }
char* ntc_data_buffer(ntc_data_t* d) noexcept { return reinterpret_cast<char*>(d->v.data()); }
uint16_t ntc_data_get_size(const ntc_data_t* d) noexcept { return static_cast<uint16_t>(d->v.size()); }
void ntc_data_resize(ntc_data_t* d, uint16_t n, ntc_error* error) noexcept
{
  ntcx::guarded([&] { d->v.resize(n); }, error);      // data.hh: bytes past the old size unset
}

// --------------------------------------------------------------------------- packet ----
ntc_packet_t* ntc_new_packet(uint16_t size) noexcept
{
  try { return new ntc_packet_t(size); } catch (...) { return nullptr; }
}
ntc_packet_t* ntc_new_packet_from(const char* src, uint16_t size) noexcept
{
  auto* p = ntc_new_packet(size);
  if (p && size) std::memcpy(p->data(), src, size);
  return p;
}
void ntc_delete_packet(ntc_packet_t* p) noexcept { delete p; }
char* ntc_packet_buffer(ntc_packet_t* p) noexcept { return reinterpret_cast<char*>(p->data()); }
uint16_t ntc_packet_get_size(const ntc_packet_t* p) noexcept { return static_cast<uint16_t>(p->size()); }
void ntc_packet_resize(ntc_packet_t* p, uint16_t n, ntc_error* error) noexcept
{
  ntcx::guarded([&] { p->v.resize(n + ntc_packet_t::shift, 0); }, error);
}

// -------------------------------------------------------------------------- encoder ----
ntc_encoder_t* ntc_new_encoder(uint8_t galois_field_size, ntc_packet_handler handler) noexcept
{
  try { return new ntc_encoder_t{ntcx::Encoder(galois_field_size, handler)}; } catch (...) { return nullptr; }
}
void ntc_delete_encoder(ntc_encoder_t* enc) noexcept { delete enc; }
void ntc_encoder_add_data(ntc_encoder_t* enc, ntc_data_t* data, ntc_error* error) noexcept
{
  ntcx::guarded([&] {
    ntcx::bytes v = std::move(data->v);
    data->v = ntcx::bytes();                       // moved-from: empty until resized
    data->v = enc->e.add_data(std::move(v));       // (with a recycled buffer's capacity)
    data->v.clear();
  }, error);
}
size_t ntc_encoder_add_packet(ntc_encoder_t* enc, ntc_packet_t* packet, ntc_error* error) noexcept
{
  return ntcx::guarded([&] {
    ntcx::bytes v = std::move(packet->v);          // the packet is left empty (moved from)
    if (v.size() < ntc_packet_t::shift) v.resize(ntc_packet_t::shift, 0);
    const size_t n = v.size() - ntc_packet_t::shift;
    return enc->e.add_packet(v.data() + ntc_packet_t::shift, n);
  }, error);
}
void ntc_encoder_generate_repair(ntc_encoder_t* enc, ntc_error* error) noexcept
{
  ntcx::guarded([&] { enc->e.generate_repair(); }, error);
}
size_t ntc_encoder_window(ntc_encoder_t* enc) noexcept { return enc->e.window(); }
void ntc_encoder_set_code_type(ntc_encoder_t* enc, ntc_code_type t) noexcept { enc->e.set_systematic(t == ntc_systematic_yes); }
void ntc_encoder_set_rate(ntc_encoder_t* enc, size_t rate) noexcept { enc->e.set_rate(rate); }
void ntc_encoder_set_window_size(ntc_encoder_t* enc, size_t size) noexcept { enc->e.set_window_size(size); }
void ntc_encoder_set_adaptive(ntc_encoder_t* enc, bool a) noexcept { enc->e.set_adaptive(a); }

// -------------------------------------------------------------------------- decoder ----
ntc_decoder_t* ntc_new_decoder(uint8_t galois_field_size, ntc_ordering_type order,
                               ntc_packet_handler ph, ntc_data_handler dh) noexcept
{
  try {
    return new ntc_decoder_t{ntcx::Decoder(galois_field_size, order == ntc_in_order_yes, ph, dh)};
  } catch (...) {
    return nullptr;
  }
}
void ntc_delete_decoder(ntc_decoder_t* dec) noexcept { delete dec; }
size_t ntc_decoder_add_packet(ntc_decoder_t* dec, ntc_packet_t* packet, ntc_error* error) noexcept
{
  return ntcx::guarded([&] {
    ntcx::bytes v = std::move(packet->v);          // the packet is left empty (moved from)
    if (v.size() < ntc_packet_t::shift) v.resize(ntc_packet_t::shift, 0);
    const size_t n = v.size() - ntc_packet_t::shift;
    return dec->d.add_packet(v.data() + ntc_packet_t::shift, n, &v);
  }, error);
}
void ntc_decoder_generate_ack(ntc_decoder_t* dec, ntc_error* error) noexcept
{
  ntcx::guarded([&] { dec->d.generate_ack(); }, error);
}
void ntc_decoder_set_ack_period(ntc_decoder_t* dec, size_t period) noexcept { dec->d.set_ack_period(period); }
void ntc_decoder_set_ack_nb_packets(ntc_decoder_t* dec, uint16_t nb) noexcept { dec->d.set_ack_nb_packets(nb); }

// ---------------------------------------------------------------- extensions (ext.h) ----
size_t ntc_encoder_counter(const ntc_encoder_t* enc, int which) noexcept { return enc->e.counter(which); }
size_t ntc_decoder_counter(const ntc_decoder_t* dec, int which) noexcept { return dec->d.counter(which); }

ntc_batch_t* ntc_new_batch(void) noexcept
{
  try { return new ntc_batch_t{}; } catch (...) { return nullptr; }
}
void ntc_delete_batch(ntc_batch_t* b) noexcept { delete b; }
void ntc_encoder_set_batch(ntc_encoder_t* enc, ntc_batch_t* b, ntc_error* error) noexcept
{
  ntcx::guarded([&] { enc->e.set_batch(b ? &b->b : nullptr); }, error);
}
void ntc_decoder_set_batch(ntc_decoder_t* dec, ntc_batch_t* b, ntc_error* error) noexcept
{
  ntcx::guarded([&] { dec->d.set_batch(b ? &b->b : nullptr); }, error);
}
void ntc_batch_set_eager(ntc_batch_t* b, int on) noexcept
{
  if (b) b->b.eager = on != 0;
}
void ntc_batch_set_async(ntc_batch_t* b, int on) noexcept
{
  if (b) b->b.async = on != 0;
}

void ntc_batch_flush(ntc_batch_t* b, ntc_error* error) noexcept
{
  ntcx::guarded([&] { b->b.flush(); }, error);
}
size_t ntc_batch_pending(const ntc_batch_t* b) noexcept { return b->b.pending(); }

void ntc_decoder_maybe_ack(ntc_decoder_t* dec, ntc_error* error) noexcept
{
  ntcx::guarded([&] { dec->d.maybe_ack(); }, error);
}

int ntc_gf_combine_host(uint32_t w, size_t n, const char* const* in, const uint16_t* lens,
                        const uint32_t* coefs, size_t out_len, char* out, int add,
                        ntc_error* error) noexcept
{
  ntc_error local{ntc_no_error, nullptr};
  ntc_error* err = error ? error : &local;
  return ntcx::guarded([&]() -> int {
    const ntcx::Field f(w);                       // rejects w outside {4, 8, 16, 32}
    (void)f;
    if (out_len > 0xFFFF) throw std::invalid_argument("region longer than 65535 bytes");
    std::vector<const uint8_t*> ins;
    std::vector<uint16_t> ls;
    std::vector<uint32_t> cs;
    if (add) {                                    // out ^= sum: out itself is a term (staged first)
      ins.push_back(reinterpret_cast<const uint8_t*>(out));
      ls.push_back(static_cast<uint16_t>(out_len));
      cs.push_back(1);
    }
    for (size_t i = 0; i < n; ++i) {
      ins.push_back(reinterpret_cast<const uint8_t*>(in[i]));
      ls.push_back(static_cast<uint16_t>(std::min<size_t>(lens[i], out_len)));
      cs.push_back(coefs[i]);
    }
    if (out_len) ntcx::Device::get().combine(w, ins.size(), ins.data(), ls.data(), cs.data(), out_len,
                                            reinterpret_cast<uint8_t*>(out));
    return 0;
  }, err) == 0 && err->type == ntc_no_error ? 0 : -1;
}

int ntc_gf_combine_rows_host(uint32_t w, size_t n, const char* const* in, const uint16_t* lens,
                             size_t rows, const uint32_t* coefs, size_t out_len, char* const* out,
                             ntc_error* error) noexcept
{
  ntc_error local{ntc_no_error, nullptr};
  ntc_error* err = error ? error : &local;
  return ntcx::guarded([&]() -> int {
    const ntcx::Field f(w);
    (void)f;
    if (out_len > 0xFFFF) throw std::invalid_argument("region longer than 65535 bytes");
    if (rows == 0 || out_len == 0) return 0;
    std::vector<uint8_t*> outs(rows);
    for (size_t s = 0; s < rows; ++s) outs[s] = reinterpret_cast<uint8_t*>(out[s]);
    ntcx::Device::get().combine_rows(w, n, reinterpret_cast<const uint8_t* const*>(in), lens, rows,
                                     coefs, out_len, outs.data());
    return 0;
  }, err) == 0 && err->type == ntc_no_error ? 0 : -1;
}

}  // extern "C"
