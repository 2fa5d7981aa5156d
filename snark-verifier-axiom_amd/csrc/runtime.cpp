#include "runtime.hpp"

#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <thread>

namespace sv {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
}
const char* last_error() { return g_err; }

namespace {
struct DevicePool {
  int device = 0;
  std::mutex mu;
  std::vector<Workspace*> free_list;
};
std::once_flag g_once;
int g_init_rc = SV_ERR_DEVICE;
std::vector<DevicePool*> g_pools;
std::mutex g_init_mu;
}  // namespace

int Workspace::reserve(size_t bytes) {
  used = 0;
  if (bytes <= cap) return SV_OK;
  SV_HIP(hipSetDevice(device));
  if (buf) {
    SV_TRY(quiesce());
    SV_HIP(hipFree(buf));
    buf = nullptr;
    cap = 0;
  }
  size_t want = bytes + bytes / 8;  // headroom for the next, slightly larger call
  hipError_t e = hipMalloc(&buf, want);
  if (e != hipSuccess) {
    e = hipMalloc(&buf, bytes);
    want = bytes;
  }
  if (e != hipSuccess) {
    buf = nullptr;
    set_error("workspace hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e));
    return SV_ERR_OOM;
  }
  cap = want;
  return SV_OK;
}

int Workspace::reserve_pinned(size_t bytes) {
  if (bytes <= pinned_cap) return SV_OK;
  if (pinned) SV_HIP(hipHostFree(pinned));
  pinned = nullptr;
  pinned_cap = 0;
  SV_HIP(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
  pinned_cap = bytes;
  return SV_OK;
}

int Workspace::reserve_in(size_t bytes) {
  if (bytes <= in_cap) return SV_OK;
  SV_HIP(hipSetDevice(device));
  if (inbuf) {
    SV_TRY(quiesce());  // a DMA of an earlier (failed) call may still target inbuf
    SV_HIP(hipFree(inbuf));
    inbuf = nullptr;
    in_cap = 0;
  }
  if (hipMalloc(&inbuf, bytes) != hipSuccess) {
    inbuf = nullptr;
    set_error("input buffer hipMalloc(%zu) failed", bytes);
    return SV_ERR_OOM;
  }
  in_cap = bytes;
  return SV_OK;
}

// Gather staging of sv_bn254_g1_msm_refs: pinned.  (Measured round 3 at 2^20, shuffled refs:
// pinned 3.00 ms, pageable staging through the runtime's own copy path 5.4 ms, pinned non-coherent
// 5.3 ms.)  The staging is read by DMAs queued on the copy stream of a DIFFERENT workspace (the
// MSM's, leased in msm_run_impl), so this workspace's streams say nothing about them.  The
// invariant that makes freeing / reusing it safe: msm_run_fed drains its copy stream before it
// returns (its Drain guard, on every exit path), and api.cpp releases the staging lease only after
// msm_run_fed has returned -- so no DMA can read a staging buffer once its lease is back in the pool.
int Workspace::reserve_stage(size_t bytes) {
  if (bytes <= stage_cap) return SV_OK;
  if (stage) SV_HIP(hipHostFree(stage));
  stage = nullptr;
  stage_cap = 0;
  SV_HIP(hipHostMalloc(&stage, bytes, hipHostMallocDefault));
  stage_cap = bytes;
  return SV_OK;
}

int Workspace::quiesce() {
  SV_HIP(hipSetDevice(device));
  if (stream) SV_HIP(hipStreamSynchronize(stream));
  if (copy_stream) SV_HIP(hipStreamSynchronize(copy_stream));
  if (sort_stream) SV_HIP(hipStreamSynchronize(sort_stream));
  return SV_OK;
}

struct Workspace::Helper {
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool pending = false, busy = false;
};

int Workspace::run_helper(std::function<void()> job) {
  if (!helper) {
    // `helper` is published only once its thread runs: if the thread cannot be created, no later
    // call queues a job that nothing would ever run (msm_run_impl's wait_stage would spin forever)
    Helper* h = new Helper();
    const int dev = device;
    try {
      std::thread([h, dev] {
        (void)hipSetDevice(dev);
        for (;;) {
          std::function<void()> j;
          {
            std::unique_lock<std::mutex> lk(h->mu);
            h->cv.wait(lk, [h] { return h->pending; });
            j = std::move(h->job);
            h->pending = false;
          }
          try {
            j();  // jobs report their own failures; nothing may escape the thread
          } catch (...) {
          }
          {
            std::lock_guard<std::mutex> lk(h->mu);
            h->busy = false;
          }
          h->cv.notify_all();
        }
      }).detach();  // lives with the pooled workspace, for the process
    } catch (const std::exception& e) {
      delete h;
      set_error("workspace helper thread: %s", e.what());
      return SV_ERR_DEVICE;
    }
    helper = h;
  }
  {
    std::lock_guard<std::mutex> lk(helper->mu);
    helper->job = std::move(job);
    helper->pending = true;
    helper->busy = true;
  }
  helper->cv.notify_all();
  return SV_OK;
}

void Workspace::wait_helper() {
  if (!helper) return;
  std::unique_lock<std::mutex> lk(helper->mu);
  helper->cv.wait(lk, [this] { return !helper->busy; });
}

int Workspace::ensure_sort_stream() {
  if (sort_stream) return SV_OK;
  SV_HIP(hipSetDevice(device));
  SV_HIP(hipStreamCreateWithFlags(&sort_stream, hipStreamNonBlocking));
  return SV_OK;
}

int Workspace::ensure_copy_stream() {
  if (copy_stream) return SV_OK;
  SV_HIP(hipSetDevice(device));
  SV_HIP(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
  return SV_OK;
}

int runtime_init(int num_devices) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (!g_pools.empty()) return SV_OK;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    set_error("no usable GPU (hipGetDeviceCount: %s, count=%d)", hipGetErrorString(e), count);
    return SV_ERR_DEVICE;
  }
  // SVGPU_DEVICE_MAP=a,b,...: logical device i runs on HIP device map[i] (repeats allowed).  With
  // "0,0,0,0,0,0,0,0" the multi-device host paths (one host thread per logical device, each with
  // its own workspace and streams, partials folded on the host) run 8-wide on one physical GPU.
  std::vector<int> map;
  if (const char* e = getenv("SVGPU_DEVICE_MAP")) {
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const long d = strtol(q, &end, 10);
      if (end == q || d < 0 || d >= count) {
        set_error("SVGPU_DEVICE_MAP=\"%s\": bad entry (HIP devices 0..%d)", e, count - 1);
        return SV_ERR_ARG;
      }
      map.push_back((int)d);
      q = *end == ',' ? end + 1 : end;
      if (*end && *end != ',') {
        set_error("SVGPU_DEVICE_MAP=\"%s\": expected comma-separated device ordinals", e);
        return SV_ERR_ARG;
      }
    }
  } else {
    for (int d = 0; d < count; d++) map.push_back(d);
  }
  if (map.empty()) {
    set_error("SVGPU_DEVICE_MAP is empty");
    return SV_ERR_ARG;
  }
  if (num_devices > 0 && (size_t)num_devices < map.size()) map.resize(num_devices);
  for (int d : map) {
    // logical devices on the same HIP device share its workspace pool (each call leases its own)
    DevicePool* p = nullptr;
    for (auto* q : g_pools)
      if (q->device == d) p = q;
    if (!p) {
      p = new DevicePool();
      p->device = d;
    }
    g_pools.push_back(p);
  }
  return SV_OK;
}

int runtime_device_count() {
  std::lock_guard<std::mutex> lk(g_init_mu);
  return (int)g_pools.size();
}

int runtime_device_id(int idx) { return g_pools[idx]->device; }

static DevicePool* pool_for(int device) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  for (auto* p : g_pools)
    if (p->device == device) return p;
  return nullptr;
}

WsLease::WsLease(int device, hipStream_t user_stream) {
  if (runtime_device_count() == 0 && runtime_init(0) != SV_OK) return;
  DevicePool* pool = pool_for(device);
  if (!pool) {
    set_error("device %d not initialised", device);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(pool->mu);
    if (!pool->free_list.empty()) {
      ws_ = pool->free_list.back();
      pool->free_list.pop_back();
    }
  }
  if (hipSetDevice(device) != hipSuccess) {
    set_error("hipSetDevice(%d) failed", device);
    if (ws_) {
      std::lock_guard<std::mutex> lk(pool->mu);
      pool->free_list.push_back(ws_);
      ws_ = nullptr;
    }
    return;
  }
  if (!ws_) {
    ws_ = new Workspace();
    ws_->device = device;
    if (hipStreamCreateWithFlags(&ws_->own_stream, hipStreamNonBlocking) != hipSuccess) {
      set_error("hipStreamCreate failed on device %d", device);
      delete ws_;
      ws_ = nullptr;
      return;
    }
    for (auto& ev : ws_->ev)
      if (hipEventCreate(&ev) != hipSuccess) {
        set_error("hipEventCreate failed on device %d", device);
        delete ws_;  // (its streams and events leak: a device that cannot create events is unusable)
        ws_ = nullptr;
        return;
      }
  }
  ws_->stream = user_stream ? user_stream : ws_->own_stream;
}

WsLease::~WsLease() {
  if (!ws_) return;
  DevicePool* pool = pool_for(ws_->device);
  std::lock_guard<std::mutex> lk(pool->mu);
  pool->free_list.push_back(ws_);
}

}  // namespace sv
