// Microbenchmark: issue rate of the integer instructions of a Montgomery product on gfx950.
//   pure v_mad_u64_u32 (8 independent 64-bit accumulators), the field.hpp pair
//   v_mad_u64_u32 + v_addc_co_u32 (carry out collected), v_mul_lo_u32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void k_mad_pure(uint64_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8];
  uint32_t a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = tid + j; a[j] = tid * 3 + j; b[j] = tid ^ (j * 77); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j]) : "v"(a[j]), "v"(b[j]) : "s0", "s1");
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j];
  out[tid] = s;
}

__global__ void k_mad_addc(uint64_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8];
  uint32_t ovf[8], a[8], b[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = tid + j; ovf[j] = 0; a[j] = tid * 3 + j; b[j] = tid ^ (j * 77); }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                   : "+v"(acc[j]), "+v"(ovf[j]) : "v"(a[j]), "v"(b[j]) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j] + ovf[j];
  out[tid] = s;
}

__global__ void k_mullo(uint64_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[8], y = tid | 1;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = tid + j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[tid] = s;
}

template <typename K>
static int run(const char* name, K kern, uint64_t* d, int insts_per_iter) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 16384, bs = 256, iters = 2000;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(bs), 0, 0, d, 10);
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
  const double lane_ops = (double)blocks * bs * iters * 8 * insts_per_iter;
  printf("%-14s %8.3f ms  %6.1f lane-op/clk/CU at 2.4 GHz (64 = one per lane-slot)\n", name, best,
         lane_ops / (best * 1e-3) / 2.4e9 / 256);
  return 0;
}

int main() {
  void* d;
  CK(hipMalloc(&d, 64 << 20));
  run("mad_pure", k_mad_pure, (uint64_t*)d, 1);
  run("mad+addc", k_mad_addc, (uint64_t*)d, 1);  // counted per (mad, addc) pair
  run("mul_lo_u32", k_mullo, (uint64_t*)d, 1);
  return 0;
}
