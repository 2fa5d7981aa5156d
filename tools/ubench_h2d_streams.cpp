// Host->device copy rate of the host-fed MSM's 96 MB (2^20 points x (64 B base + 32 B scalar)) as
// one copy or split over 2 / 4 streams issued back to back (each stream may get its own SDMA
// engine), from pageable memory (the caller's arrays, what sv_bn254_g1_msm copies from) and from
// pinned memory.  Round 5, VERDICT r04 item 5: is one copy stream below the link rate?
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_h2d_streams.cpp -o tools/ubench_h2d_streams
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t bytes = (size_t)96 << 20;
  char* dev;
  CK(hipMalloc(&dev, bytes));
  std::vector<char> pageable(bytes);
  for (size_t i = 0; i < bytes; i += 4096) pageable[i] = (char)i;
  char* pinned;
  CK(hipHostMalloc(&pinned, bytes, hipHostMallocDefault));
  memcpy(pinned, pageable.data(), bytes);
  hipStream_t st[4];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (int src = 0; src < 2; src++) {
    const char* h = src ? pinned : pageable.data();
    for (int ns : {1, 2, 4}) {
      double best = 1e30;
      for (int rep = 0; rep < 6; rep++) {
        CK(hipDeviceSynchronize());
        const double t0 = now_ms();
        const size_t part = bytes / ns;
        for (int k = 0; k < ns; k++) CK(hipMemcpyAsync(dev + k * part, h + k * part, part, hipMemcpyHostToDevice, st[k]));
        for (int k = 0; k < ns; k++) CK(hipStreamSynchronize(st[k]));
        const double t = now_ms() - t0;
        if (rep > 0 && t < best) best = t;
      }
      printf("%-8s %d stream(s): %.3f ms  %.1f GB/s\n", src ? "pinned" : "pageable", ns, best, bytes / best / 1e6);
    }
  }
  return 0;
}
