// Microbenchmark (round 5): does v_mad_u64_u32 leave issue slots for other VALU instructions on
// gfx950?  Each kernel runs 8 independent v_mad_u64_u32 accumulator chains per iteration and, in
// the mixed variants, N other VALU instructions per mad on their own registers (no dependence on
// the mads).  If a mixed variant takes the time of the pure one, those instructions co-issue beside
// the mads; if it takes the sum, every VALU instruction costs issue time.
// Occupancy: blocks of 256 threads, launch bounds (256, 4) -> 4 waves per SIMD, as k_accumulate.
// Usage: ./ubench_issue
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);          \
      return 1;                                                                \
    }                                                                          \
  } while (0)

// OP: 0 none, 1 v_add_u32, 2 v_and_b32, 3 v_lshrrev_b64, 4 v_mul_lo_u32, 5 v_lshl_add_u64,
//     6 v_add_co/v_addc pair (counted as 2), 7 v_bfe_u32
template <int OP, int N>
__global__ void __launch_bounds__(256, 4) k_mix(uint64_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8], w[8];
  uint32_t a[8], b[8], x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    acc[j] = tid + j;
    a[j] = tid * 3 + j;
    b[j] = tid ^ (j * 77);
    x[j] = tid * 7 + j;
    w[j] = (uint64_t)tid << 20 | j;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j]) : "v"(a[j]), "v"(b[j]) : "s0", "s1");
#pragma unroll
      for (int r = 0; r < N; r++) {
        const int k = (j + r) & 7;
        if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(a[k]));
        if constexpr (OP == 2) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[k]) : "v"(b[k]));
        if constexpr (OP == 3) asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(w[k]));
        if constexpr (OP == 4) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(b[k]));
        if constexpr (OP == 5) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(w[k]) : "v"(w[(k + 1) & 7]));
        if constexpr (OP == 6)
          asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %2, vcc, 0, %2, vcc"
                       : "+v"(x[k]), "+v"(a[(k + 3) & 7]) : "v"(b[k]) : "vcc");
        if constexpr (OP == 7) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(x[k]));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j] + x[j] + w[j] + a[j];
  out[tid] = s;
}

// no mads: NA independent v_add_u32 per iteration (the VALU issue rate of a plain 32-bit op), or
// 16 independent mad chains (is 8 chains x 4 waves enough to reach the mad issue rate?)
template <int MODE>
__global__ void __launch_bounds__(256, 4) k_alt(uint64_t* out, int iters) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[16];
  uint32_t a[16], x[16];
#pragma unroll
  for (int j = 0; j < 16; j++) {
    acc[j] = tid + j;
    a[j] = tid * 3 + j;
    x[j] = tid * 7 + j;
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if constexpr (MODE == 0) {
        asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a[j]));
      } else {
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j]) : "v"(a[j]), "v"(x[j]) : "s0", "s1");
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j + 8]) : "v"(a[j + 8]), "v"(x[j + 8]) : "s0", "s1");
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 16; j++) s += acc[j] + x[j];
  out[tid] = s;
}

// dependent-chain latency at ONE wave per SIMD (the decider's occupancy): C independent
// v_mad_u64_u32 chains per iteration; cycles per iteration / C = the issue cost once C chains
// cover the latency, cycles per iteration = the latency of one dependent mad while C = 1
template <int C, int ADDC>
__global__ void __launch_bounds__(64) k_lat(uint64_t* out, int iters, unsigned long long* cyc) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[C];
  uint32_t a[C], b[C], o[C];
#pragma unroll
  for (int j = 0; j < C; j++) {
    acc[j] = tid + j;
    a[j] = tid * 3 + j;
    b[j] = tid ^ (j * 77);
    o[j] = 0;
  }
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int j = 0; j < C; j++) {
      if constexpr (ADDC)
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                     : "+v"(acc[j]), "+v"(o[j]) : "v"(a[j]), "v"(b[j]) : "vcc");
      else
        asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j]) : "v"(a[j]), "v"(b[j]) : "s0", "s1");
    }
  }
  const unsigned long long t1 = clock64();
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < C; j++) s += acc[j] + o[j];
  out[tid] = s;
  if (tid == 0) *cyc = t1 - t0;
}
template <int C, int ADDC>
static void lat(const char* name, uint64_t* d, unsigned long long* dc) {
  const int iters = 4096;
  hipLaunchKernelGGL((k_lat<C, ADDC>), dim3(1), dim3(64), 0, 0, d, 16, dc);
  hipLaunchKernelGGL((k_lat<C, ADDC>), dim3(1), dim3(64), 0, 0, d, iters, dc);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("one wave, %-24s %2d chain(s): %6.2f cycles per iteration, %5.2f per instruction group\n", name, C,
         (double)c / iters, (double)c / iters / C);
}

// single-wave issue interval of one instruction type: 8 independent chains per iteration, 16
// iterations unrolled per loop trip (loop overhead / 128), one block of T threads (T = 64: one wave
// on one SIMD; T = 512: two waves per SIMD)
// OP: 0 v_mad_u64_u32, 1 v_add_u32, 2 v_add_co_u32 + v_addc_co_u32 (one pair), 3 v_mul_lo_u32,
//     4 v_perm_b32, 5 v_add_u32_dpp (row_ror:4), 6 v_mov_b32_dpp + v_add_u32 (pair)
template <int OP>
__global__ void __launch_bounds__(512) k_one(uint64_t* out, int iters, unsigned long long* cyc) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc[8];
  uint32_t a[8], b[8], x[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    acc[j] = tid + j;
    a[j] = tid * 3 + j;
    b[j] = tid ^ (j * 77);
    x[j] = tid * 7 + j;
  }
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < 16; u++) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if constexpr (OP == 0) asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[j]) : "v"(a[j]), "v"(b[j]) : "s0", "s1");
        if constexpr (OP == 1) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[j]) : "v"(a[j]));
        if constexpr (OP == 2)
          asm volatile("v_add_co_u32 %0, vcc, %0, %2\n\tv_addc_co_u32 %1, vcc, 0, %1, vcc"
                       : "+v"(x[j]), "+v"(a[j]) : "v"(b[j]) : "vcc");
        if constexpr (OP == 3) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[j]) : "v"(b[j]));
        if constexpr (OP == 4) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[j]) : "v"(b[j]), "v"(a[j]));
        if constexpr (OP == 5) asm volatile("v_add_u32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(x[j]));
        if constexpr (OP == 6)
          asm volatile("v_mov_b32_dpp %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\ts_nop 1\n\tv_add_u32 %0, %0, %1"
                       : "+v"(x[j]), "+v"(a[j]));
      }
    }
  }
  const unsigned long long t1 = clock64();
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j] + x[j] + a[j];
  out[tid] = s;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
template <int OP>
static void one(const char* name, uint64_t* d, unsigned long long* dc) {
  const int iters = 256;
  for (int T : {64, 512}) {
    hipLaunchKernelGGL(k_one<OP>, dim3(1), dim3(T), 0, 0, d, 4, dc);
    hipLaunchKernelGGL(k_one<OP>, dim3(1), dim3(T), 0, 0, d, iters, dc);
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    printf("%-28s %s: %6.2f cycles per instruction (group) per wave\n", name,
           T == 64 ? "1 wave / SIMD " : "2 waves / SIMD", (double)c / (iters * 128.0));
  }
}

template <typename K>
static float run(const char* name, K kern, uint64_t* d, double others_per_mad, float base) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 8192, bs = 256, iters = 1000;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(bs), 0, 0, d, 10);
  if (hipDeviceSynchronize() != hipSuccess) return -1.f;
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(bs), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  const double waves = (double)blocks * bs / 64, mads = waves * iters * 8;
  // SIMD-cycles per wave-instruction at 2.4 GHz over 1024 SIMDs
  const double simd_cycles = best * 1e-3 * 2.4e9 * 1024;
  printf("%-22s %8.3f ms  mad lane-op/clk/CU %6.1f  cycles per mad %5.2f  extra vs pure %+6.2f cycles per other op\n",
         name, best, mads * 64 / (best * 1e-3) / 2.4e9 / 256, simd_cycles / mads,
         others_per_mad > 0 ? (best - base) * 1e-3 * 2.4e9 * 1024 / (mads * others_per_mad) : 0.0);
  return best;
}

int main() {
  void* d;
  CK(hipMalloc(&d, 64 << 20));
  const float base = run("mad only", k_mix<0, 0>, (uint64_t*)d, 0, 0);
  run("mad + 1 add_u32", k_mix<1, 1>, (uint64_t*)d, 1, base);
  run("mad + 2 add_u32", k_mix<1, 2>, (uint64_t*)d, 2, base);
  run("mad + 4 add_u32", k_mix<1, 4>, (uint64_t*)d, 4, base);
  run("mad + 1 and_b32", k_mix<2, 1>, (uint64_t*)d, 1, base);
  run("mad + 1 lshrrev_b64", k_mix<3, 1>, (uint64_t*)d, 1, base);
  run("mad + 1 mul_lo_u32", k_mix<4, 1>, (uint64_t*)d, 1, base);
  run("mad + 1 lshl_add_u64", k_mix<5, 1>, (uint64_t*)d, 1, base);
  run("mad + 1 add_co/addc", k_mix<6, 1>, (uint64_t*)d, 2, base);
  run("mad + 1 bfe_u32", k_mix<7, 1>, (uint64_t*)d, 1, base);
  run("mad + 8 add_u32", k_mix<1, 8>, (uint64_t*)d, 8, base);
  // per 'mad' slot below: k_alt<0> issues 8 adds per iteration (reported as 'mads'), k_alt<1> 16 mads
  run("add_u32 only (as mads)", k_alt<0>, (uint64_t*)d, 0, 0);
  const float m16 = run("16 mad chains (x2)", k_alt<1>, (uint64_t*)d, 0, 0);
  printf("16 mad chains: %.2f cycles per mad\n", m16 * 1e-3 * 2.4e9 * 1024 / (8192.0 * 256 / 64 * 1000 * 16));
  unsigned long long* dc;
  CK(hipMalloc(&dc, 8));
  lat<1, 0>("mad", (uint64_t*)d, dc);
  lat<2, 0>("mad", (uint64_t*)d, dc);
  lat<4, 0>("mad", (uint64_t*)d, dc);
  lat<8, 0>("mad", (uint64_t*)d, dc);
  lat<1, 1>("mad + addc (vcc)", (uint64_t*)d, dc);
  lat<2, 1>("mad + addc (vcc)", (uint64_t*)d, dc);
  lat<4, 1>("mad + addc (vcc)", (uint64_t*)d, dc);
  one<0>("v_mad_u64_u32", (uint64_t*)d, dc);
  one<1>("v_add_u32", (uint64_t*)d, dc);
  one<2>("v_add_co + v_addc (pair)", (uint64_t*)d, dc);
  one<3>("v_mul_lo_u32", (uint64_t*)d, dc);
  one<4>("v_perm_b32", (uint64_t*)d, dc);
  one<5>("v_add_u32_dpp row_ror", (uint64_t*)d, dc);
  one<6>("v_mov_dpp + v_add (pair)", (uint64_t*)d, dc);
  return 0;
}
