// Per-operation latency of the workgroup decider's Fq12 ops (csrc/decider.hip namespace wg) on one
// 256-thread block: w_sqr / w_mul / w_frob in a dependent loop, timed with clock64 on the device.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -Isnark-verifier-axiom_amd/csrc tools/ubench_wg.hip \
//          snark-verifier-axiom_amd/csrc/runtime.cpp -o tools/ubench_wg
#include "../snark-verifier-axiom_amd/csrc/decider.hip"
#include "../snark-verifier-axiom_amd/csrc/field29.hpp"

#include <cstdio>
#include <vector>

using namespace sv;

__global__ void __launch_bounds__(256) k_bench(int op, int iters, unsigned long long* cycles, uint32_t* sink) {
  __shared__ Fq2 S[3 * 6];
  __shared__ Fq gam[3 * 6 * 2];
  const int t = threadIdx.x;
  if (t < 6) {
    S[t] = Fq2::one();
    S[t].c1 = Fq::one();
    S[6 + t] = S[t];
  }
  for (int i = t; i < 3 * 6 * 16; i += 256) reinterpret_cast<uint32_t*>(gam)[i] = c_gamma[i];
  __syncthreads();
  Fq2* a = S;
  Fq2* b = S + 6;
  Fq2* c = S + 12;
  const wg::WLane L = wg::wlane_init();
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if (op == 0) wg::w_sqr(L, c, a);
    else if (op == 1) wg::w_mul(L, c, a, b);
    else if (op == 2) wg::w_frob(L, c, a, 1, gam);
    else wg::w_conj(c, a);
    Fq2* tmp = a;
    a = c;
    c = tmp;
  }
  const unsigned long long t1 = clock64();
  if (t == 0) {
    *cycles = t1 - t0;
    sink[0] = a[0].c0.v[0];
  }
}

// one operation per kernel (no op switch in the loop): OP as k_bench's op
template <int OP>
__global__ void __launch_bounds__(256) k_bench1(int iters, unsigned long long* cycles, uint32_t* sink) {
  __shared__ Fq2 S[3 * 6];
  __shared__ Fq gam[3 * 6 * 2];
  const int t = threadIdx.x;
  if (t < 6) {
    S[t] = Fq2::one();
    S[t].c1 = Fq::one();
    S[6 + t] = S[t];
  }
  for (int i = t; i < 3 * 6 * 16; i += 256) reinterpret_cast<uint32_t*>(gam)[i] = c_gamma[i];
  __syncthreads();
  Fq2* a = S;
  Fq2* b = S + 6;
  Fq2* c = S + 12;
  const wg::WLane L = wg::wlane_init();
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if constexpr (OP == 0) wg::w_sqr(L, c, a);
    else if constexpr (OP == 1) wg::w_mul(L, c, a, b);
    else wg::w_frob(L, c, a, 1, gam);
    Fq2* tmp = a;
    a = c;
    c = tmp;
  }
  const unsigned long long t1 = clock64();
  if (t == 0) {
    *cycles = t1 - t0;
    sink[0] = a[0].c0.v[0];
  }
}

// round 5: a product on 8 x 32-bit words computed with field29.hpp's mul_ilp (x R' domain: the words
// are converted to 9 x 29-bit limbs and back) -- timing only, the domain is not the slots' one
__device__ __forceinline__ Fq mul29w(const Fq& a, const Fq& b) {
  const r29::F x = r29::from_words(a.v), y = r29::from_words(b.v);
  Fq r;
  r29::to_words(r29::mul_ilp(x, y), r.v);
  return r;
}

// w_mul with parts switched off (mode bits): 1 no product, 2 no lane sum, 4 no lz_reduce,
// 8 no barrier, 16 no LDS operand loads (registers instead), 32 the product by mul29w; the same
// code as wg::w_mul otherwise
__device__ __forceinline__ void w_mul_dbg(const wg::WLane& L, Fq2* __restrict__ dst, const Fq2* a, const Fq2* b,
                                          int mode) {
  using namespace wg;
  const int t = threadIdx.x;
  if (t < 192) {
    const int q = L.mq;
    Fq ax, by;
    if (mode & 16) {
      ax = Fq::one();
      ax.v[0] ^= t;
      by = ax;
    } else {
      ax = ld_fq((q & 1) ? &a[L.mi].c1 : &a[L.mi].c0);
      by = ld_fq((q == 1 || q == 2) ? &b[L.mjj].c1 : &b[L.mjj].c0);
    }
    Fq v = (mode & 1) ? ax : ((mode & 32) ? mul29w(ax, by) : fe_mul_lazy(ax, by));
    if (!L.mact) v = Fq::zero();
    const Fq nv = fq_neg2p(v);
    Lz re, im;
    place(lz(q == 1 ? nv : v), lz(q == 1 ? v : nv), q >= 2, L.mwrap, re, im);
    const Lz s = (mode & 2) ? re : lane_sum<5>(re, im);
    const int j = t & 31;
    if (j < 2) {
      Fq r;
      if (mode & 4) {
        for (int x = 0; x < 8; x++) r.v[x] = s.v[x];
      } else {
        r = lz_reduce(s);
      }
      st_fq(j ? &dst[L.mk].c1 : &dst[L.mk].c0, r);
    }
  }
  if (!(mode & 8)) __syncthreads();
}

// the same switches over round 5's w_mul (lane_sum24): 1 no product, 2 no cross-lane levels (the
// lane's own split, multiply and normalisation only), 4 no lz_reduce, 8 no barrier, 16 no LDS
// operand loads; mode bit 64 selects this variant in k_bench_dbg
__device__ __forceinline__ void w_mul_dbg24(const wg::WLane& L, Fq2* __restrict__ dst, const Fq2* a, const Fq2* b,
                                            int mode) {
  using namespace wg;
  const int t = threadIdx.x;
  if (t < 192) {
    const int q = L.mq;
    Fq ax, by;
    if (mode & 16) {
      ax = Fq::one();
      ax.v[0] ^= t;
      by = ax;
    } else {
      ax = ld_fq((q & 1) ? &a[L.mi].c1 : &a[L.mi].c0);
      by = ld_fq((q == 1 || q == 2) ? &b[L.mjj].c1 : &b[L.mjj].c0);
    }
    const Fq v = (mode & 1) ? ax : fe_mul_lazy(ax, by);
    Lz s;
    if (mode & 2) {
      uint32_t l[kL24], x[kL24];
      split24(v, l);
#pragma unroll
      for (int i = 0; i < kL24; i++) x[i] = L.mkeep * l[i] + L.msend * l[i];
      s = norm24(x);
    } else {
      s = lane_sum24<5>(v, L.mkeep, L.msend);
    }
    const int j = t & 31;
    if (j < 2) {
      Fq r;
      if (mode & 4) {
        for (int x = 0; x < 8; x++) r.v[x] = s.v[x];
      } else {
        r = lz_reduce(s);
      }
      st_fq(j ? &dst[L.mk].c1 : &dst[L.mk].c0, r);
    }
  }
  if (!(mode & 8)) __syncthreads();
}

__global__ void __launch_bounds__(256) k_bench_dbg(int mode, int iters, unsigned long long* cycles, uint32_t* sink) {
  __shared__ Fq2 S[3 * 6];
  const int t = threadIdx.x;
  if (t < 6) {
    S[t] = Fq2::one();
    S[6 + t] = S[t];
  }
  __syncthreads();
  Fq2* a = S;
  Fq2* b = S + 6;
  Fq2* c = S + 12;
  const wg::WLane L = wg::wlane_init();
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if (mode & 64) w_mul_dbg24(L, c, a, b, mode);
    else w_mul_dbg(L, c, a, b, mode);
    Fq2* tmp = a;
    a = c;
    c = tmp;
  }
  const unsigned long long t1 = clock64();
  if (t == 0) {
    *cycles = t1 - t0;
    sink[0] = a[0].c0.v[0];
  }
}

__global__ void k_fqmul(int iters, unsigned long long* cycles, uint32_t* sink) {
  Fq x = Fq::one();
  x.v[0] ^= threadIdx.x;
  const Fq y = x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = x * y;
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) *cycles = t1 - t0;
  sink[threadIdx.x] = x.v[0];
}

__global__ void k_fqmul_var(int var, int iters, unsigned long long* cycles, uint32_t* sink) {
  Fq x = Fq::one();
  x.v[0] ^= threadIdx.x;
  const Fq y = x;
  const unsigned long long t0 = clock64();
  if (var == 0)
    for (int i = 0; i < iters; i++) x = fe_mul_lazy(x, y);
  else
    for (int i = 0; i < iters; i++) x = mul29w(x, y);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) *cycles = t1 - t0;
  sink[threadIdx.x] = x.v[0];
}

// one lane inverting in Fq2 (the decider's w_norm_inv), dependent chain
__global__ void k_inv(int iters, unsigned long long* cycles, uint32_t* sink) {
  Fq2 x = Fq2::one();
  x.c1 = Fq::one();
  x.c0.v[0] ^= threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) x = fq2_inv(x);
  const unsigned long long t1 = clock64();
  if (threadIdx.x == 0) *cycles = t1 - t0;
  sink[threadIdx.x] = x.c0.v[0];
}

// every CU busy (grid = CU count) with the w_sqr loop: shader clock = d(memtime) / d(memrealtime) x 100 MHz
__global__ void __launch_bounds__(256) k_clock(int iters, unsigned long long* out) {
  __shared__ Fq2 S[2 * 6];
  const int t = threadIdx.x;
  if (t < 6) {
    S[t] = Fq2::one();
    S[t].c1 = Fq::one();
  }
  __syncthreads();
  Fq2* a = S;
  Fq2* c = S + 6;
  const wg::WLane L = wg::wlane_init();
  const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; i++) {
    wg::w_sqr(L, c, a);
    Fq2* tmp = a;
    a = c;
    c = tmp;
  }
  const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (t == 0) {
    out[3 * blockIdx.x] = c1 - c0;
    out[3 * blockIdx.x + 1] = r1 - r0;
    out[3 * blockIdx.x + 2] = a[0].c0.v[0];
  }
}

int main() {
  unsigned long long* dc;
  uint32_t* ds;
  (void)hipMalloc(&dc, 8);
  (void)hipMalloc(&ds, 4096);
  const char* names[] = {"w_sqr", "w_mul", "w_frob", "w_conj"};
  const int iters = 200;
  for (int op = 0; op < 4; op++) {
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, op, 4, dc, ds);
    hipLaunchKernelGGL(k_bench, dim3(1), dim3(256), 0, 0, op, iters, dc, ds);
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    printf("%-7s %8.1f cycles/op (clock64)\n", names[op], (double)c / iters);
  }
  {
    void (*ks[3])(int, unsigned long long*, uint32_t*) = {k_bench1<0>, k_bench1<1>, k_bench1<2>};
    for (int op = 0; op < 3; op++) {
      hipLaunchKernelGGL(ks[op], dim3(1), dim3(256), 0, 0, 4, dc, ds);
      hipLaunchKernelGGL(ks[op], dim3(1), dim3(256), 0, 0, iters, dc, ds);
      unsigned long long c = 0;
      (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
      printf("%-7s %8.1f cycles/op (alone in its kernel)\n", names[op], (double)c / iters);
    }
  }
  for (int mode : {0, 1, 2, 4, 8, 16, 64, 64 | 1, 64 | 2, 64 | 4, 64 | 8, 64 | 16, 64 | 1 | 2 | 4, 64 | 1 | 2 | 4 | 8, 64 | 31}) {
    hipLaunchKernelGGL(k_bench_dbg, dim3(1), dim3(256), 0, 0, mode, 4, dc, ds);
    hipLaunchKernelGGL(k_bench_dbg, dim3(1), dim3(256), 0, 0, mode, iters, dc, ds);
    unsigned long long c = 0;
    (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    printf("w_mul mode %2d %8.1f cycles/op\n", mode, (double)c / iters);
  }
  hipLaunchKernelGGL(k_fqmul, dim3(1), dim3(64), 0, 0, iters, dc, ds);
  unsigned long long c = 0;
  (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("%-7s %8.1f cycles/op (one wave, dependent Fq products)\n", "fq_mul", (double)c / iters);
  for (int var = 0; var < 2; var++) {
    hipLaunchKernelGGL(k_fqmul_var, dim3(1), dim3(64), 0, 0, var, 4, dc, ds);
    hipLaunchKernelGGL(k_fqmul_var, dim3(1), dim3(64), 0, 0, var, iters, dc, ds);
    (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
    printf("%-12s %8.1f cycles/op (one wave, dependent)\n", var ? "mul29w" : "fe_mul_lazy", (double)c / iters);
  }
  hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, 2, dc, ds);
  hipLaunchKernelGGL(k_inv, dim3(1), dim3(64), 0, 0, 20, dc, ds);
  (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
  printf("%-7s %8.1f cycles/op (one lane, dependent Fq2 inversions)\n", "fq2_inv", (double)c / 20);
  for (int grid : {1, 256}) {
    unsigned long long* dk;
    (void)hipMalloc(&dk, 3 * 8 * grid);
    std::vector<unsigned long long> h(3 * grid);
    hipLaunchKernelGGL(k_clock, dim3(grid), dim3(256), 0, 0, 2000, dk);
    hipLaunchKernelGGL(k_clock, dim3(grid), dim3(256), 0, 0, 2000, dk);
    (void)hipMemcpy(h.data(), dk, 3 * 8 * grid, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int b = 0; b < grid; b++) cyc += h[3 * b], rt += h[3 * b + 1];
    printf("grid %3d: w_sqr %7.1f cycles/op, shader clock %.0f MHz, %.3f us/op\n", grid, cyc / grid / 2000,
           cyc / rt * 100.0, rt / grid / 2000 / 100.0);
    (void)hipFree(dk);
  }
  return 0;
}
