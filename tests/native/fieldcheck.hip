// Test-only device harness for the fused field primitives of csrc/field.hpp / csrc/curve.hpp
// (fe_sqr_hp, fe_mul_sum<N>, mul_diff): their inline-asm device paths differ from the host
// build (which falls back to a*a and separate products), so tests/test_gpu_field_edges.py runs
// them on the GPU over edge operands (0, 1, p-1, p-2, 2^k, all-ones low limbs, ...) and checks
// them against Python big-int Montgomery arithmetic.  Not part of libsvgpu.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "curve.hpp"
#include "field.hpp"

using namespace sv;

enum { OP_MUL = 0, OP_SQR_HP = 1, OP_SUM1 = 2, OP_SUM2 = 3, OP_SUM3 = 4, OP_MUL_DIFF = 5 };

template <class M>
__device__ Fe<M> ld(const uint32_t* p) {
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = p[i];
  return r;
}

template <class M>
__global__ void k_fieldcheck(int op, const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d,
                             uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<M> x = ld<M>(a + 8 * i), y = ld<M>(b + 8 * i), z = ld<M>(c + 8 * i), w = ld<M>(d + 8 * i);
  Fe<M> r = Fe<M>::zero();
  if (op == OP_MUL) {
    r = x * y;
  } else if (op == OP_SQR_HP) {
    r = fe_sqr_hp(x);
  } else if (op == OP_SUM1) {
    const Fe<M> u[1] = {x}, v[1] = {y};
    r = fe_mul_sum(u, v);
  } else if (op == OP_SUM2) {
    const Fe<M> u[2] = {x, z}, v[2] = {y, w};
    r = fe_mul_sum(u, v);
  } else if (op == OP_SUM3) {
    const Fe<M> u[3] = {x, z, y}, v[3] = {y, w, z};
    r = fe_mul_sum(u, v);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) out[8 * i + k] = r.v[k];
}

__global__ void k_fieldcheck_diff(const uint32_t* a, const uint32_t* b, const uint32_t* c, const uint32_t* d,
                                  uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fq r = mul_diff(ld<FqTag>(a + 8 * i), ld<FqTag>(b + 8 * i), ld<FqTag>(c + 8 * i), ld<FqTag>(d + 8 * i));
#pragma unroll
  for (int k = 0; k < 8; k++) out[8 * i + k] = r.v[k];
}

// field: 0 = Fq, 1 = Fr.  Buffers are host arrays of n elements (8 x u32 LE limbs each).
// Returns 0 on success, the hipError_t otherwise.
extern "C" int fc_run(int op, int field, const void* a, const void* b, const void* c, const void* d, void* out,
                      size_t n) {
  if (n == 0) return 0;
  const size_t bytes = n * 32;
  uint32_t* dev = nullptr;
  hipError_t e = hipMalloc(&dev, 5 * bytes);
  if (e != hipSuccess) return (int)e;
  const void* src[4] = {a, b, c, d};
  for (int k = 0; k < 4 && e == hipSuccess; k++) e = hipMemcpy(dev + k * 8 * n, src[k], bytes, hipMemcpyHostToDevice);
  uint32_t* o = dev + 32 * n;
  const dim3 grid((unsigned)((n + 255) / 256)), blk(256);
  if (e == hipSuccess) {
    if (op == OP_MUL_DIFF)
      hipLaunchKernelGGL(k_fieldcheck_diff, grid, blk, 0, 0, dev, dev + 8 * n, dev + 16 * n, dev + 24 * n, o,
                         (uint32_t)n);
    else if (field == 0)
      hipLaunchKernelGGL(k_fieldcheck<FqTag>, grid, blk, 0, 0, op, dev, dev + 8 * n, dev + 16 * n, dev + 24 * n, o,
                         (uint32_t)n);
    else
      hipLaunchKernelGGL(k_fieldcheck<FrTag>, grid, blk, 0, 0, op, dev, dev + 8 * n, dev + 16 * n, dev + 24 * n, o,
                         (uint32_t)n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpy(out, o, bytes, hipMemcpyDeviceToHost);
  (void)hipFree(dev);
  return (int)e;
}
