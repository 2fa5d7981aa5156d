// Host->device staging microbenchmark for the host-buffer MSM entry point (sv_bn254_g1_msm):
// how fast can 96 B/point of caller-owned PAGEABLE memory reach HBM?
//   a) hipMemcpy straight from pageable memory (the runtime stages it itself)
//   b) pinned ring: T host threads memcpy chunks into pinned slots, DMA each slot asynchronously
//   c) hipHostRegister the caller's buffer, DMA, unregister
//   d) pinned -> device DMA alone (the PCIe ceiling)
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_h2d.cpp -o tools/ubench_h2d -lpthread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  size_t mb = argc > 1 ? atoi(argv[1]) : 96;
  size_t bytes = mb << 20;
  char* host = (char*)malloc(bytes);
  for (size_t i = 0; i < bytes; i += 4096) host[i] = (char)i;
  memset(host, 1, bytes);
  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int reps = 5;
  auto report = [&](const char* name, double ms) {
    printf("%-44s %8.3f ms  %7.1f GB/s\n", name, ms, bytes / ms / 1e6);
  };

  // a) pageable
  CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
  double t0 = now_ms();
  for (int r = 0; r < reps; r++) CK(hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice));
  report("a) hipMemcpy pageable", (now_ms() - t0) / reps);
  t0 = now_ms();
  for (int r = 0; r < reps; r++) CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st));
  CK(hipStreamSynchronize(st));
  report("a') hipMemcpyAsync pageable", (now_ms() - t0) / reps);

  // d) pinned ceiling
  char* pin = nullptr;
  CK(hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault));
  memcpy(pin, host, bytes);
  CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, st));
  CK(hipStreamSynchronize(st));
  t0 = now_ms();
  for (int r = 0; r < reps; r++) CK(hipMemcpyAsync(dev, pin, bytes, hipMemcpyHostToDevice, st));
  CK(hipStreamSynchronize(st));
  report("d) pinned DMA only", (now_ms() - t0) / reps);

  // host memcpy bandwidth with T threads (pageable -> pinned)
  for (int T : {1, 2, 4, 8, 16}) {
    t0 = now_ms();
    for (int r = 0; r < reps; r++) {
      std::vector<std::thread> th;
      size_t per = (bytes + T - 1) / T;
      for (int k = 0; k < T; k++)
        th.emplace_back([&, k] {
          size_t lo = k * per, hi = std::min(bytes, lo + per);
          if (lo < hi) memcpy(pin + lo, host + lo, hi - lo);
        });
      for (auto& t : th) t.join();
    }
    char name[64];
    snprintf(name, sizeof name, "memcpy pageable->pinned T=%d", T);
    report(name, (now_ms() - t0) / reps);
  }

  // b) pinned ring: T threads fill chunk slots; each slot is DMAed as soon as it is full
  for (size_t chunk_mb : {4, 8, 16}) {
    for (int T : {4, 8, 16}) {
      const size_t chunk = chunk_mb << 20;
      const int slots = 4;
      std::vector<hipEvent_t> ev(slots);
      for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      double best = 1e9;
      for (int r = 0; r < reps; r++) {
        t0 = now_ms();
        size_t nch = (bytes + chunk - 1) / chunk;
        for (size_t c = 0; c < nch; c++) {
          int s = c % slots;
          if (c >= (size_t)slots) CK(hipEventSynchronize(ev[s]));
          size_t lo = c * chunk, len = std::min(chunk, bytes - lo);
          char* dst = pin + (size_t)s * chunk;
          std::vector<std::thread> th;
          size_t per = (len + T - 1) / T;
          for (int k = 0; k < T; k++)
            th.emplace_back([&, k] {
              size_t a = k * per, b = std::min(len, a + per);
              if (a < b) memcpy(dst + a, host + lo + a, b - a);
            });
          for (auto& t : th) t.join();
          CK(hipMemcpyAsync((char*)dev + lo, dst, len, hipMemcpyHostToDevice, st));
          CK(hipEventRecord(ev[s], st));
        }
        CK(hipStreamSynchronize(st));
        best = std::min(best, now_ms() - t0);
      }
      char name[64];
      snprintf(name, sizeof name, "b) pinned ring chunk=%zuMB T=%d (spawn/chunk)", chunk_mb, T);
      report(name, best);
      for (auto& e : ev) CK(hipEventDestroy(e));
    }
  }

  // b2) pinned ring with persistent workers: each worker owns every T-th chunk
  for (size_t chunk_mb : {2, 4, 8}) {
    for (int T : {4, 8, 16}) {
      const size_t chunk = chunk_mb << 20;
      const size_t nch = (bytes + chunk - 1) / chunk;
      double best = 1e9;
      for (int r = 0; r < reps; r++) {
        t0 = now_ms();
        std::atomic<size_t> next{0};
        std::vector<std::thread> th;
        std::vector<hipStream_t> ss(T);
        for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        double t1 = now_ms();
        for (int k = 0; k < T; k++)
          th.emplace_back([&, k] {
            for (size_t c; (c = next.fetch_add(1)) < nch;) {
              size_t lo = c * chunk, len = std::min(chunk, bytes - lo);
              memcpy(pin + lo, host + lo, len);  // full-size pinned staging (no slot reuse)
              CK(hipMemcpyAsync((char*)dev + lo, pin + lo, len, hipMemcpyHostToDevice, ss[k]));
            }
          });
        for (auto& t : th) t.join();
        for (auto& s : ss) CK(hipStreamSynchronize(s));
        double el = now_ms() - t1;
        for (auto& s : ss) CK(hipStreamDestroy(s));
        (void)t0;
        best = std::min(best, el);
      }
      char name[64];
      snprintf(name, sizeof name, "b2) workers chunk=%zuMB T=%d", chunk_mb, T);
      report(name, best);
    }
  }

  // c) register the caller's buffer
  t0 = now_ms();
  for (int r = 0; r < reps; r++) {
    CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
    void* dp = nullptr;
    CK(hipHostGetDevicePointer(&dp, host, 0));
    CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    CK(hipHostUnregister(host));
  }
  report("c) hipHostRegister + DMA + unregister", (now_ms() - t0) / reps);
  t0 = now_ms();
  for (int r = 0; r < reps; r++) {
    CK(hipHostRegister(host, bytes, hipHostRegisterDefault));
    CK(hipHostUnregister(host));
  }
  report("c') register + unregister only", (now_ms() - t0) / reps);
  printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
  return 0;
}
