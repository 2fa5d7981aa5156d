#include "runtime.hpp"
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
using namespace sv;
struct Fe { uint64_t l[4]; };
struct Af { Fe x, y; };
struct Ref { const Fe* s; const Af* b; };
int main() {
  size_t n = 1 << 20;
  std::vector<Fe> S(n); std::vector<Af> B(n); std::vector<Ref> R(n);
  for (size_t i = 0; i < n; i++) { S[i].l[0] = i; B[i].x.l[0] = i; R[i] = {&S[i], &B[i]}; }
  std::vector<Fe> hs(n); std::vector<Af> hb(n);
  for (int rep = 0; rep < 3; rep++) {
    auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < 4; k++) {
      size_t a = n * k / 4, b = n * (k + 1) / 4;
      host_parallel_for(b - a, 8192, [&](size_t x, size_t y) { for (size_t i = a + x; i < a + y; i++) hs[i] = *R[i].s; });
      host_parallel_for(b - a, 8192, [&](size_t x, size_t y) { for (size_t i = a + x; i < a + y; i++) hb[i] = *R[i].b; });
    }
    auto t1 = std::chrono::steady_clock::now();
    printf("threads %d: %.3f ms\n", host_threads(), std::chrono::duration<double, std::milli>(t1 - t0).count());
  }
}
