// Round 6: the host-fed MSM's eight pageable copies (2^20 points, pieces 5,4,4,3 of 16: each
// piece's 32-B scalars then its 64-B bases) issued back to back by ONE thread on one stream (as the
// MSM's feeder does) against TWO threads on two streams (scalars on one, bases on the other, so
// one copy's setup overlaps the other's transfer).  Prints the best of 8 runs of each.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_h2d_pieces.cpp -o tools/bin/ubench_h2d_pieces
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
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
  const size_t n = (size_t)1 << 20;
  const size_t sb = n * 32, bb = n * 64;
  char *ds, *db;
  CK(hipMalloc(&ds, sb));
  CK(hipMalloc(&db, bb));
  std::vector<char> hs(sb), hb(bb);
  for (size_t i = 0; i < sb; i += 4096) hs[i] = (char)i;
  for (size_t i = 0; i < bb; i += 4096) hb[i] = (char)i;
  const int w[4] = {5, 4, 4, 3};
  size_t lo[5] = {0};
  for (int k = 0; k < 4; k++) lo[k + 1] = k == 3 ? n : lo[k] + (n * w[k] / 16 & ~(size_t)1023);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  for (int mode = 0; mode < 2; mode++) {
    double best = 1e30;
    for (int rep = 0; rep < 9; rep++) {
      CK(hipDeviceSynchronize());
      const double t0 = now_ms();
      if (mode == 0) {
        for (int k = 0; k < 4; k++) {
          CK(hipMemcpyAsync(ds + lo[k] * 32, hs.data() + lo[k] * 32, (lo[k + 1] - lo[k]) * 32, hipMemcpyHostToDevice, s0));
          CK(hipMemcpyAsync(db + lo[k] * 64, hb.data() + lo[k] * 64, (lo[k + 1] - lo[k]) * 64, hipMemcpyHostToDevice, s0));
        }
        CK(hipStreamSynchronize(s0));
      } else {
        std::thread th([&] {
          for (int k = 0; k < 4; k++)
            CK(hipMemcpyAsync(ds + lo[k] * 32, hs.data() + lo[k] * 32, (lo[k + 1] - lo[k]) * 32, hipMemcpyHostToDevice, s1));
          CK(hipStreamSynchronize(s1));
        });
        for (int k = 0; k < 4; k++)
          CK(hipMemcpyAsync(db + lo[k] * 64, hb.data() + lo[k] * 64, (lo[k + 1] - lo[k]) * 64, hipMemcpyHostToDevice, s0));
        CK(hipStreamSynchronize(s0));
        th.join();
      }
      const double t = now_ms() - t0;
      if (rep > 0 && t < best) best = t;
    }
    printf("%s: %.3f ms  %.1f GB/s\n", mode ? "two threads, two streams" : "one thread, one stream  ", best,
           (sb + bb) / best / 1e6);
  }
  return 0;
}
