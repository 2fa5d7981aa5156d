// Microbenchmark (round 4): Montgomery product over 9 x 29-bit limbs (R = 2^261) against the
// library's 8 x 32-bit product-scanning product (field.hpp fe_mul_lazy).
// With 29-bit limbs every partial product is below 2^58 and a column of 18 of them plus the carry
// stays below 2^63: each partial product is ONE v_mad_u64_u32 into a 64-bit accumulator, with no
// carry add (the 32-bit form needs a v_addc per partial product).  Same lazy contract as
// fe_mul_lazy: inputs below 2p give a result below 2p (4p < R).
// Host: `./ubench_r29 check` prints (a, b, a*b/R mod p) triples for tools/check_r29.py;
// device: throughput of both products, 4 independent chains per thread.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstring>

#include "../snark-verifier-axiom_amd/csrc/field.hpp"

#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

namespace r29 {
constexpr uint32_t MASK = (1u << 29) - 1;
constexpr uint32_t NP = 0x4866389u;  // -p^-1 mod 2^29
__host__ __device__ constexpr uint32_t P(int i) {
  constexpr uint32_t p[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                             0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
  return p[i];
}
struct F {
  uint32_t v[9];
};
__host__ __device__ __forceinline__ uint64_t mad(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}
__host__ __device__ __forceinline__ F mul(const F& a, const F& b) {
  uint32_t m[9];
  F t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc = mad(a.v[i], b.v[j], acc);
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 9) acc = mad(m[i], P(j), acc);
    }
    if (k < 9) {
      m[k] = ((uint32_t)acc * NP) & MASK;
      acc = mad(m[k], P(0), acc);
    } else {
      t.v[k - 9] = (uint32_t)acc & MASK;
    }
    acc >>= 29;
  }
  t.v[8] = (uint32_t)acc;
  return t;
}
}  // namespace r29

template <int C>
__global__ void __launch_bounds__(256) k_r29(uint32_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  r29::F x[C], y;
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int i = 0; i < 9; i++) x[c].v[i] = ((tid * 2654435761u) ^ (i * 40503u + c)) & (i == 8 ? 0x3fffffu : r29::MASK);
#pragma unroll
  for (int i = 0; i < 9; i++) y.v[i] = ((tid * 97u) + i * 13u) & (i == 8 ? 0x3fffffu : r29::MASK);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < C; c++) x[c] = r29::mul(x[c], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int i = 0; i < 9; i++) s ^= x[c].v[i];
  out[tid] = s;
}

template <int C>
__global__ void __launch_bounds__(256) k_r32(uint32_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  sv::Fq x[C], y;
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int i = 0; i < 8; i++) x[c].v[i] = ((tid * 2654435761u) ^ (i * 40503u + c)) & (i == 7 ? 0x0fffffffu : ~0u);
#pragma unroll
  for (int i = 0; i < 8; i++) y.v[i] = ((tid * 97u) + i * 13u) & (i == 7 ? 0x0fffffffu : ~0u);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < C; c++) x[c] = sv::fe_mul_lazy(x[c], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < C; c++)
#pragma unroll
    for (int i = 0; i < 8; i++) s ^= x[c].v[i];
  out[tid] = s;
}

template <typename K>
static int run(const char* name, K kern, uint32_t* d, int chains) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 4096, bs = 256, iters = 400;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(bs), 0, 0, d, 4);
  CK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(bs), 0, 0, d, iters);
    hipEventRecord(e1);
    CK(hipEventSynchronize(e1));
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double prods = (double)blocks * bs * iters * chains;
  printf("%-22s %8.3f ms  %7.1f G products/s\n", name, best, prods / (best * 1e-3) / 1e9);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "check")) {  // host: triples for tools/check_r29.py
    uint64_t s = 0x1234567;
    for (int n = 0; n < 200; n++) {
      r29::F a, b;
      for (int i = 0; i < 9; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        a.v[i] = (uint32_t)(s >> 33) & r29::MASK;
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        b.v[i] = (uint32_t)(s >> 33) & r29::MASK;
      }
      a.v[8] &= 0x3fffffu;  // below 2^254 < 2p
      b.v[8] &= 0x3fffffu;
      r29::F r = r29::mul(a, b);
      for (const r29::F* f : {&a, &b, &r}) {
        for (int i = 8; i >= 0; i--) printf("%08x%s", f->v[i], i ? "," : "");
        printf(f == &r ? "\n" : " ");
      }
    }
    return 0;
  }
  uint32_t* d;
  CK(hipMalloc(&d, 16 << 20));
  run("r32 fe_mul_lazy x4", k_r32<4>, d, 4);
  run("r29 mul x4", k_r29<4>, d, 4);
  run("r32 fe_mul_lazy x2", k_r32<2>, d, 2);
  run("r29 mul x2", k_r29<2>, d, 2);
  return 0;
}
