#include "hostpool.hpp"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace sv {

namespace {
// Fixed pool of host workers; one job at a time (concurrent callers queue on job_mu_).  A job is
// split into one slice per thread, claimed dynamically; workers spin for a while after each job
// before sleeping, because the host-fed MSM issues its gather jobs in bursts (a futex wake-up
// costs about as much as a whole slice, so sleeping workers left the caller doing every slice).
//
// Claims are tied to the job: claim_ packs (job generation, slice count, next slice) into ONE
// atomic word, published by the caller with a release store AFTER the job's function and size
// and the reset of done_.  A worker claims slice k by a CAS of that word from (g, parts, k) to
// (g, parts, k + 1), so a straggler still looping on job g can never take a slice of job g + 1
// (its CAS fails once the word holds g + 1), and it reads fn_ / n_ only after a successful claim:
// job g cannot complete before that slice's done_ increment, so the fields it reads are job g's.
class HostPool {
 public:
  // slice count and next-slice index are at most kMaxThreads (parts <= nthreads_), so 11 bits each
  // leave 42 bits of job generation: a wrap needs 2^42 jobs (~10^11 host-fed calls at ~12 jobs
  // each), i.e. a straggler would have to stall across 4e12 jobs to see its generation again
  static constexpr int kMaxThreads = 1024;
  static constexpr uint64_t kIdxBits = 11, kIdxMask = (uint64_t(1) << kIdxBits) - 1;
  static_assert((uint64_t(1) << kIdxBits) > (uint64_t)kMaxThreads, "slice index must hold nthreads_");
  static_assert(64 - 2 * kIdxBits >= 40, "job generation needs >= 40 bits");
  using Fn = std::function<void(size_t, size_t)>;

  HostPool() {
    int hw = (int)std::thread::hardware_concurrency();
    nthreads_ = hw > 16 ? 16 : (hw > 0 ? hw : 1);
    if (const char* e = getenv("SVGPU_HOST_THREADS")) nthreads_ = atoi(e) > 0 ? atoi(e) : 1;
    if (nthreads_ > kMaxThreads) nthreads_ = kMaxThreads;
    for (int i = 1; i < nthreads_; i++) workers_.emplace_back([this] { loop(); });
    for (auto& w : workers_) w.detach();  // the pool lives for the process
  }
  int threads() const { return nthreads_; }

  void run(size_t n, size_t grain, const Fn& fn) {
    if (n == 0) return;
    size_t parts = (n + grain - 1) / (grain ? grain : 1);
    if (parts > (size_t)nthreads_) parts = (size_t)nthreads_;
    if (parts <= 1) {
      fn(0, n);
      return;
    }
    std::lock_guard<std::mutex> job(job_mu_);
    // the previous job is complete (its caller saw done_ == parts under job_mu_): every one of its
    // claims has been made, so nothing reads or writes these fields until the word below changes
    done_.store(0, std::memory_order_relaxed);
    fn_.store(&fn, std::memory_order_relaxed);
    n_.store(n, std::memory_order_relaxed);
    const uint64_t g = ++gen_;  // job_mu_ held
    {
      std::lock_guard<std::mutex> lk(mu_);
      claim_.store((g << (2 * kIdxBits)) | ((uint64_t)parts << kIdxBits), std::memory_order_release);
    }
    // wake only the workers the job can use (a 2-slice job -- the accumulation's two MSMs -- used
    // to wake all 15, each then spinning ~1 ms for a next job: CPU the calling thread's serial work,
    // e.g. create_proof's host sponge, competes with under the box's CPU quota); workers still
    // spinning from a burst see the new word without a wake-up
    for (size_t k = 1; k < parts; k++) cv_.notify_one();
    work();
    while (done_.load(std::memory_order_acquire) < parts) std::this_thread::yield();
  }

 private:
  static uint64_t gen_of(uint64_t w) { return w >> (2 * kIdxBits); }

  void work() {
    for (;;) {
      uint64_t w = claim_.load(std::memory_order_acquire);
      size_t k, parts;
      for (;;) {
        k = (size_t)(w & kIdxMask);
        parts = (size_t)((w >> kIdxBits) & kIdxMask);
        if (k >= parts) return;  // every slice of the current job is taken
        if (claim_.compare_exchange_weak(w, w + 1, std::memory_order_acq_rel, std::memory_order_acquire)) break;
      }
      const Fn* fn = fn_.load(std::memory_order_relaxed);
      const size_t n = n_.load(std::memory_order_relaxed);
      (*fn)(n * k / parts, n * (k + 1) / parts);
      done_.fetch_add(1, std::memory_order_acq_rel);
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      // spin ~1 ms for the next job of a burst, then sleep
      auto t0 = std::chrono::steady_clock::now();
      while (gen_of(claim_.load(std::memory_order_acquire)) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(1))
        std::this_thread::yield();
      if (gen_of(claim_.load(std::memory_order_acquire)) == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_of(claim_.load(std::memory_order_acquire)) != seen; });
      }
      seen = gen_of(claim_.load(std::memory_order_acquire));
      work();
    }
  }

  int nthreads_ = 1;
  std::vector<std::thread> workers_;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_;
  uint64_t gen_ = 0;  // last published job (job_mu_)
  std::atomic<const Fn*> fn_{nullptr};
  std::atomic<size_t> n_{0}, done_{0};
  std::atomic<uint64_t> claim_{0};
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

}  // namespace sv
