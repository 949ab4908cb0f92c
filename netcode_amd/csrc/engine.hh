// engine.hh -- engine state and helpers shared by the engine's translation units
// (ntc_gf256.hip: reference-schedule encode/decode + MAC kernels; ntc_dense.hip: dense codes).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

#include "netcode/gpu.h"

struct ntc_gf256_engine {
  int device = 0;
  size_t plan_cap_G = 0, plan_cap_k = 0, plan_cap_rp = 0;
  uint16_t* plan_m = nullptr;
  uint16_t* plan_in = nullptr;
  uint16_t* plan_out = nullptr;
  uint8_t* plan_coef = nullptr;
  void* enc_coef = nullptr;
  size_t enc_coef_cap = 0;
  // encode generation pairing (short symbols, continuous ids): per generation 0 = alone,
  // 1 = shares its MAC wave with generation g + 255 (equal coefficient matrices), 2 = that partner
  void* enc_pair = nullptr;
  size_t enc_pair_cap = 0;
  // split-k MAC partial outputs (launch_mac, few tasks) and the device's CU count
  void* kout = nullptr;
  size_t kout_cap = 0;
  uint32_t ncu = 0;
  // bit-sliced copy of a tall encode / combine's sources (launch_mac, bs_preslice)
  void* slice = nullptr;
  size_t slice_cap = 0;
  // the last plan also wrote the decode MAC's input row addresses (row_ptr) for these buffers
  const uint8_t* rows_src = nullptr;
  const uint8_t* rows_rep = nullptr;
  uint32_t rows_stride = 0;
  void* row_ptr = nullptr;     // bit-sliced decode: input row address per plan position
  size_t row_ptr_cap = 0;
  int mac_kind = NTC_GF256_MAC_AUTO;
  int pair_j = 2;                   // gf_mac_bsp sources per wave and turn (NTC_GF256_PAIRJ)
  int pair_sets = 3;                // gf_mac_bsp slot sets, 3 or 4 (NTC_GF256_PAIRSETS)
  uint32_t rowtile_force = 0;  // bit-sliced row tile 8 or 16 (NTC_GF256_ROWTILE; 0 = by rows)
  uint32_t ksplit_force = 0;   // split-k part count 1..8 (NTC_GF256_KSPLIT; 0 = the heuristic)
  int slice_force = -1;        // pre-sliced sources 0 / 1 (NTC_GF256_SLICE; -1 = by rows)
  int plan_kind = NTC_GF256_PLAN_AUTO;
  // MAC kernel timing (ntc_gf256_set_timing): events bracket the last encode / decode MAC launch
  bool timing = false;
  hipEvent_t mac_ev[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
  // kernel timing log (ntc_gf256_timing_log): an event pair around every launch, in launch order
  uint32_t tlog_cap = 0, tlog_n = 0;
  uint32_t tlog_mask = ~0u;            // bit k: log kernels of kind k (ntc_gf256_timing_kinds)
  std::vector<hipEvent_t> tlog_ev;     // 2 per entry
  std::vector<uint32_t> tlog_kind;     // NTC_GF256_K_*
  // geometry of the last plan (decode_apply must match)
  uint32_t last_G = 0, last_k = 0, last_r = 0, last_rp = 0;
  // dense-code workspace (ntc_dense.hip): augmented matrices (ping-pong), panel trackers,
  // pivot rows, row flags, combine coefficients
  void* dn_x = nullptr;   size_t dn_x_cap = 0;
  void* dn_y = nullptr;   size_t dn_y_cap = 0;
  void* dn_w = nullptr;   size_t dn_w_cap = 0;
  void* dn_piv = nullptr; size_t dn_piv_cap = 0;
  void* dn_flag = nullptr; size_t dn_flag_cap = 0;
  void* dn_coef = nullptr; size_t dn_coef_cap = 0;
  void* dn_ok = nullptr;  size_t dn_ok_cap = 0;
  // Graph capture: once any launch of this engine has been captured (KernelTimer notes it), a
  // growing workspace buffer is retired here instead of freed -- a captured graph keeps the old
  // address -- and released with the engine.
  bool captured_any = false;
  std::vector<void*> retired;
};

namespace ntcgpu {

// Record `msg` as this thread's last error (ntc_gf256_last_error) and return `code`.
int fail(int code, const std::string& msg);
// NTC_GPU_OK, or the mapped status with the HIP error text recorded.
int hip_check(hipError_t e, const char* what);
// Grow a device buffer of engine `e` to at least `need` bytes (contents not preserved; the old
// buffer is freed, or retired if a graph may hold it: captured_any).
int ensure_buf(ntc_gf256_engine* e, void** p, size_t* cap, size_t need, const char* what);
// Release a workspace buffer that is being replaced (freed, or retired after a capture).
void drop_buf(ntc_gf256_engine* e, void* p);
// Allocation size for a workspace buffer of capacity cap that must hold need bytes (doubling once
// any launch has been captured, so that few outgrown buffers are retired).
size_t grow_to(const ntc_gf256_engine* e, size_t need, size_t cap);
// Coefficient rows padded to the MAC kernels' row tile (ntc_gf256_coef_pitch).
uint32_t tile_rp(uint32_t r);

// Scope guard around one kernel launch (or a sequence of launches) for the timing log.
// Single kernels are launched with hipExtLaunchKernelGGL(..., kt.start(), kt.stop(), 0, ...):
// the dispatch itself stamps the event pair (ext = true), so timing every kernel adds no packets
// between them.  A multi-launch region (ext = false) is bracketed by event records on the stream
// instead: the start before the first launch, the end when the scope closes.
class KernelTimer {
 public:
  KernelTimer(ntc_gf256_engine* e, uint32_t kind, hipStream_t st, bool ext = false)
      : e_(e), st_(st), ext_(ext)
  {
    // every launch region passes here: note a graph capture (the null stream is never captured,
    // so the default-stream case costs no runtime call)
    if (!e_->captured_any && st_ != nullptr) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st_, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
        e_->captured_any = true;
    }
    if (e_->tlog_n < e_->tlog_cap && ((e_->tlog_mask >> kind) & 1u)) {
      slot_ = static_cast<int>(e_->tlog_n++);
      e_->tlog_kind[slot_] = kind;
      if (!ext_) (void)hipEventRecord(e_->tlog_ev[2 * slot_], st_);
    }
  }
  ~KernelTimer()
  {
    if (slot_ >= 0 && !ext_) (void)hipEventRecord(e_->tlog_ev[2 * slot_ + 1], st_);
  }
  // the events an ext launch hands to the dispatch (nullptr: not logged)
  hipEvent_t start() const { return slot_ >= 0 && ext_ ? e_->tlog_ev[2 * slot_] : nullptr; }
  hipEvent_t stop() const { return slot_ >= 0 && ext_ ? e_->tlog_ev[2 * slot_ + 1] : nullptr; }
  KernelTimer(const KernelTimer&) = delete;
  KernelTimer& operator=(const KernelTimer&) = delete;

 private:
  ntc_gf256_engine* e_;
  hipStream_t st_;
  bool ext_;
  int slot_ = -1;
};

}  // namespace ntcgpu
