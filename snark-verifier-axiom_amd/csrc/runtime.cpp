#include "runtime.hpp"

#include <cstdarg>
#include <cstdio>
#include <atomic>
#include <chrono>
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
    SV_HIP(hipStreamSynchronize(stream));
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
    SV_HIP(hipStreamSynchronize(stream));
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

int Workspace::reserve_stage(size_t bytes) {
  if (bytes <= stage_cap) return SV_OK;
  if (stage) SV_HIP(hipHostFree(stage));
  stage = nullptr;
  stage_cap = 0;
  SV_HIP(hipHostMalloc(&stage, bytes, hipHostMallocDefault));
  stage_cap = bytes;
  return SV_OK;
}

int Workspace::ensure_copy_stream() {
  if (copy_stream) return SV_OK;
  SV_HIP(hipSetDevice(device));
  SV_HIP(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
  return SV_OK;
}

namespace {
// Fixed pool of host workers; one job at a time (concurrent callers queue on job_mu).  A job is
// split into one slice per thread, claimed dynamically; workers spin for a while after each job
// before sleeping, because the host-fed MSM issues its gather jobs in bursts (a futex wake-up
// costs about as much as a whole slice, so sleeping workers left the caller doing every slice).
class HostPool {
 public:
  HostPool() {
    int hw = (int)std::thread::hardware_concurrency();
    nthreads_ = hw > 16 ? 16 : (hw > 0 ? hw : 1);
    if (const char* e = getenv("SVGPU_HOST_THREADS")) nthreads_ = atoi(e) > 0 ? atoi(e) : 1;
    for (int i = 1; i < nthreads_; i++) workers_.emplace_back([this] { loop(); });
    for (auto& w : workers_) w.detach();  // the pool lives for the process
  }
  int threads() const { return nthreads_; }
  void run(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
    if (n == 0) return;
    size_t parts = (n + grain - 1) / (grain ? grain : 1);
    if (parts > (size_t)nthreads_) parts = (size_t)nthreads_;
    if (parts <= 1) {
      fn(0, n);
      return;
    }
    std::lock_guard<std::mutex> job(job_mu_);
    fn_ = &fn;
    n_ = n;
    parts_ = parts;
    next_.store(0, std::memory_order_relaxed);
    done_.store(0, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    work();
    while (done_.load(std::memory_order_acquire) != parts_) std::this_thread::yield();
  }

 private:
  void work() {
    for (;;) {
      const size_t k = next_.fetch_add(1, std::memory_order_acq_rel);
      if (k >= parts_) return;
      (*fn_)(n_ * k / parts_, n_ * (k + 1) / parts_);
      done_.fetch_add(1, std::memory_order_acq_rel);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      // spin ~1 ms for the next job of a burst, then sleep
      auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(1))
        std::this_thread::yield();
      if (gen_.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
      }
      seen = gen_.load(std::memory_order_acquire);
      work();
    }
  }
  int nthreads_ = 1;
  std::vector<std::thread> workers_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_;
  const std::function<void(size_t, size_t)>* fn_ = nullptr;
  size_t n_ = 0, parts_ = 0;
  std::atomic<size_t> next_{0}, done_{0};
  std::atomic<uint64_t> gen_{0};
};
HostPool& host_pool() {
  static HostPool* p = new HostPool();  // leaked: detached workers outlive static destruction
  return *p;
}
}  // namespace

void host_parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn) {
  host_pool().run(n, grain, fn);
}
int host_threads() { return host_pool().threads(); }

int runtime_init(int num_devices) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (!g_pools.empty()) return SV_OK;
  int count = 0;
  hipError_t e = hipGetDeviceCount(&count);
  if (e != hipSuccess || count <= 0) {
    set_error("no usable GPU (hipGetDeviceCount: %s, count=%d)", hipGetErrorString(e), count);
    return SV_ERR_DEVICE;
  }
  if (num_devices > 0 && num_devices < count) count = num_devices;
  for (int d = 0; d < count; d++) {
    auto* p = new DevicePool();
    p->device = d;
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
    for (auto& ev : ws_->ev) hipEventCreate(&ev);
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
