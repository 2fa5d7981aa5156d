// Stress test of libsvgpu's host worker pool (csrc/hostpool.cpp), built with ThreadSanitizer by
// `make tsan-check` (CPU only, no HIP).  Several caller threads issue thousands of back-to-back
// host_parallel_for jobs whose slice counts alternate between 2 and the pool size, so workers
// still leaving one job meet the next one -- the pattern of the NativeLoader gather
// (sv_bn254_g1_msm_refs: 16-slice gathers) next to sv_bn254_kzg_accumulate's 2-slice job.
// Every job checks that each index ran exactly once and that no slice ran after the call
// returned; a watchdog turns a hang into a failure.
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <thread>
#include <vector>

#include "hostpool.hpp"

static std::atomic<long> g_late{0};

int main(int argc, char** argv) {
  const int callers = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 3000;
  alarm(300);  // a lost done_ increment would spin forever: SIGALRM ends the run as a failure
  std::atomic<long> bad{0};
  std::vector<std::thread> th;
  for (int c = 0; c < callers; c++)
    th.emplace_back([&, c] {
      std::mt19937 rng(1234 + c);
      std::vector<uint32_t> mark;
      for (int it = 0; it < iters; it++) {
        size_t n, grain;
        switch ((it + c) % 4) {
          case 0: n = 2, grain = 1; break;                     // 2 slices
          case 1: n = 16 * 64, grain = 64; break;              // a slice per pool thread
          case 2: n = 1 + rng() % 5000, grain = 1 + rng() % 700; break;
          default: n = 3 + rng() % 29, grain = 1; break;
        }
        mark.assign(n, 0);
        std::atomic<bool> returned{false};
        const uint32_t tag = (uint32_t)it + 1;
        sv::host_parallel_for(n, grain, [&](size_t lo, size_t hi) {
          if (returned.load(std::memory_order_relaxed)) g_late.fetch_add(1);
          for (size_t i = lo; i < hi; i++) mark[i] += tag;
          if (((lo ^ (size_t)it) & 7) == 0) std::this_thread::yield();  // stragglers
        });
        returned.store(true, std::memory_order_relaxed);
        for (size_t i = 0; i < n; i++)
          if (mark[i] != tag) {
            bad.fetch_add(1);
            break;
          }
      }
    });
  for (auto& t : th) t.join();
  printf("pool_stress: threads=%d callers=%d jobs=%ld bad=%ld late=%ld\n", sv::host_threads(), callers,
         (long)callers * iters, bad.load(), g_late.load());
  return bad.load() || g_late.load() ? 1 : 0;
}
