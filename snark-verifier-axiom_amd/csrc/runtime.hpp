// libsvgpu runtime: per-device stream/workspace pools, error reporting, HIP error plumbing.
// Calls are re-entrant (SURVEY.md section 8b "Threading"): every call acquires its own
// Workspace (stream + grow-only device buffer + events) from the device's pool.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/svgpu.h"
#include "hostpool.hpp"

namespace sv {

void set_error(const char* fmt, ...);
const char* last_error();

struct Workspace {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;  // own_stream or a caller-provided stream for this call
  char* buf = nullptr;
  size_t cap = 0;
  size_t used = 0;
  char* pinned = nullptr;  // host staging
  size_t pinned_cap = 0;
  // host-buffer entry points: pooled device copy of the caller's inputs (no per-call hipMalloc /
  // hipFree), pinned gather staging, and a copy stream that runs ahead of `stream`
  char* inbuf = nullptr;
  size_t in_cap = 0;
  char* stage = nullptr;
  size_t stage_cap = 0;
  hipStream_t copy_stream = nullptr;
  hipStream_t sort_stream = nullptr;  // host-fed MSM: piece k + 1's sort beside piece k's accumulate
  static constexpr int kEvents = 64;
  hipEvent_t ev[kEvents] = {};


  // carve `bytes` from the device buffer (256-B aligned); call reserve() first
  template <class T>
  T* carve(size_t count) {
    size_t bytes = (count * sizeof(T) + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(buf + used);
    used += bytes;
    return p;
  }
  static size_t aligned(size_t bytes) { return (bytes + 255) & ~size_t(255); }
  int reserve(size_t bytes);         // grow-only; resets `used`
  int reserve_pinned(size_t bytes);  // grow-only pinned host staging
  int reserve_in(size_t bytes);      // grow-only device input buffer
  int reserve_stage(size_t bytes);   // grow-only pinned gather staging
  int ensure_copy_stream();
  int ensure_sort_stream();
  int quiesce();
  // A persistent helper thread of this workspace (created on first use, current device set once):
  // run_helper queues `job` on it, wait_helper blocks until that job has returned.  The host-fed
  // MSM's feeder runs here (a new std::thread per call, with its first HIP call, cost ~0.2 ms).
  int run_helper(std::function<void()> job);
  void wait_helper();
  struct Helper;
  Helper* helper = nullptr;  // wait for the compute and copy streams (before freeing or reusing staging)
};

// RAII lease of a per-device workspace; stream override optional.
class WsLease {
 public:
  WsLease(int device, hipStream_t user_stream);
  ~WsLease();
  Workspace* get() { return ws_; }
  bool ok() const { return ws_ != nullptr; }

 private:
  Workspace* ws_ = nullptr;
};

int runtime_init(int num_devices);
int runtime_device_count();
int runtime_device_id(int idx);  // HIP ordinal of the idx-th initialised device

#define SV_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ::sv::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call, hipGetErrorString(e_)); \
      return e_ == hipErrorOutOfMemory ? SV_ERR_OOM : SV_ERR_DEVICE;                   \
    }                                                                                  \
  } while (0)

#define SV_TRY(expr)        \
  do {                      \
    int rc_ = (expr);       \
    if (rc_ != SV_OK) return rc_; \
  } while (0)

}  // namespace sv
