// Microbenchmark: VALU issue rates on gfx950 for the instructions a floating-point (52-bit limb)
// Montgomery product would use, next to v_mad_u64_u32 (the current 32-bit limb product).
//   v_fma_f64, v_add_f64, v_lshl_add_u64 (one-instruction 64-bit add), v_add_co_u32+v_addc_co_u32,
//   v_mad_u64_u32, v_lshrrev_b64.
// Each thread runs 8 independent chains; 16384 blocks x 256 threads fill every SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void k_fma64(double* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  double x[8];
  double y = 1.0 + 1e-9 * (tid & 7), z = 1e-7;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = tid + j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] = __builtin_fma(x[j], y, z);
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += x[j];
  out[tid] = s;
}

__global__ void k_add64f(double* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  double x[8];
  double z = 1e-7 * (tid & 3);
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = tid + j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[j]) : "v"(z));
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += x[j];
  out[tid] = s;
}

__global__ void k_lshladd(uint64_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t x[8], y = tid * 0x9E3779B97F4A7C15ull;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = tid + j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(x[j]) : "v"(y));
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[tid] = s;
}

__global__ void k_addc(uint64_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t lo[8], hi[8], ylo = tid * 2654435761u, yhi = tid ^ 0x5555u;
#pragma unroll
  for (int j = 0; j < 8; j++) { lo[j] = tid + j; hi[j] = j; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++)
      asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, %1, %3, vcc"
                   : "+v"(lo[j]), "+v"(hi[j]) : "v"(ylo), "v"(yhi) : "vcc");
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= ((uint64_t)hi[j] << 32) | lo[j];
  out[tid] = s;
}

__global__ void k_mad(uint64_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8];
  uint32_t x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) { acc[j] = tid + j; x[j] = tid * 3 + j; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) x[j] ^= (uint32_t)(acc[j] >> 40);
#pragma unroll
    for (int j = 0; j < 8; j++)
      acc[j] = (uint64_t)x[j] * x[(j + 1) & 7] + acc[j];
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j];
  out[tid] = s;
}

__global__ void k_shr64(uint64_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = (tid + j) * 0x9E3779B97F4A7C15ull;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(x[j]));
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[tid] = s;
}

__global__ void k_add32(uint32_t* out, int iters) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[8], y = tid * 2654435761u;
#pragma unroll
  for (int j = 0; j < 8; j++) x[j] = tid + j;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(y));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= x[j];
  out[tid] = s;
}

template <typename K, typename T>
static int run(const char* name, K kern, T* d, int insts_per_iter) {
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
  double lane_ops = (double)blocks * bs * iters * 8 * insts_per_iter;
  double per_clk_cu = lane_ops / (best * 1e-3) / 2.4e9 / 256;
  printf("%-16s %8.3f ms  %8.2f T lane-op/s  %6.1f lane-op/clk/CU (2.4 GHz; 64 = one per lane-slot)\n", name, best,
         lane_ops / (best * 1e-3) / 1e12, per_clk_cu);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, prop.multiProcessorCount, prop.clockRate);
  void* d;
  CK(hipMalloc(&d, 64 << 20));
  run("v_fma_f64", k_fma64, (double*)d, 1);
  run("v_add_f64", k_add64f, (double*)d, 1);
  run("v_lshl_add_u64", k_lshladd, (uint64_t*)d, 1);
  run("add_co+addc", k_addc, (uint64_t*)d, 2);
  run("v_mad_u64_u32", k_mad, (uint64_t*)d, 1);
  run("v_lshrrev_b64", k_shr64, (uint64_t*)d, 1);
  run("v_add_u32", k_add32, (uint32_t*)d, 1);
  return 0;
}
