// Batch-affine bucket accumulation, measured (round 5).
//
// k_xyzz: the library's bucket step -- each thread adds K consecutive entries of a random entry list
//   into one XYZZ accumulator with csrc/curve29.hpp's mixed addition (points as x R' words, as
//   k_accumulate reads its point table).
// k_pairs<M, INV>: the same K entries as K / 2 affine PAIR sums folded into the XYZZ accumulator:
//   per batch of M pairs, Montgomery's trick (the prefix products of the M x-differences in
//   registers, ONE inversion, the backward pass re-reading each pair's points), then per pair
//   lambda = dy / dx, x3 = lambda^2 - x0 - x1, y3 = lambda (x0 - x3) - y0 (5 products + 1 square
//   per pair), and one XYZZ mixed addition of (x3, y3).  INV = 0: a per-lane Fermat inversion
//   (255 squarings + 127 products on every lane); INV = 1: no inversion (timing of the rest only:
//   the result is wrong).  No pair has dx = 0 here (distinct points, none the negative of another);
//   a real kernel needs the doubling and cancellation cases.
// k_inv: the per-lane inversion alone.
// Points: multiples of the generator (on the curve, so sums do not depend on the addition order).
// Prints ns per entry for each, and checks k_pairs<., 0> against k_xyzz (same projective sums).
// Usage: ./ubench_affine [log2 entries = 24]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../snark-verifier-axiom_amd/csrc/curve.hpp"
#include "../snark-verifier-axiom_amd/csrc/curve29.hpp"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);            \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

using namespace sv;
constexpr uint32_t K = 32;  // entries per thread

__device__ __forceinline__ void load_xy(const uint4* __restrict__ b, uint32_t i, r29::F& x, r29::F& y) {
  const uint4 q0 = b[4 * i], q1 = b[4 * i + 1], q2 = b[4 * i + 2], q3 = b[4 * i + 3];
  const uint32_t xw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  const uint32_t yw[8] = {q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
  x = r29::from_words(xw);
  y = r29::from_words(yw);
}
__device__ __forceinline__ r29::F load_x(const uint4* __restrict__ b, uint32_t i) {
  const uint4 q0 = b[4 * i], q1 = b[4 * i + 1];
  const uint32_t xw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
  return r29::from_words(xw);
}

__device__ __forceinline__ void store_canon(const r29::Xyzz& acc, G1Xyzz* out) {
  G1Xyzz r;
  r29::to_r32(acc.X, r.X.v);
  r29::to_r32(acc.Y, r.Y.v);
  r29::to_r32(acc.ZZ, r.ZZ.v);
  r29::to_r32(acc.ZZZ, r.ZZZ.v);
  *out = r;
}

__global__ void __launch_bounds__(256) k_xyzz(const uint4* __restrict__ pts, const uint32_t* __restrict__ ent,
                                              uint32_t m, G1Xyzz* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t * K >= m) return;
  r29::Xyzz acc = r29::identity();
  for (uint32_t e = t * K; e < t * K + K; e++) {
    r29::F x, y;
    load_xy(pts, ent[e], x, y);
    acc = r29::madd(acc, x, y);
  }
  store_canon(acc, out + t);
}

// a^(p - 2) R' for a R' (binary method, exponent bits from the top; every lane the same exponent)
__device__ __forceinline__ r29::F inv_fermat(const r29::F& a) {
  constexpr uint64_t E[4] = {0x3c208c16d87cfd45ull, 0x97816a916871ca8dull, 0xb85045b68181585dull,
                             0x30644e72e131a029ull};
  r29::F r = r29::one();
#pragma unroll 1
  for (int w = 3; w >= 0; w--)
#pragma unroll 1
    for (int b = 63; b >= 0; b--) {
      r = r29::sqr(r);
      if ((E[w] >> b) & 1) r = r29::mul(r, a);
    }
  return r;
}

template <int M, int INV>
__global__ void __launch_bounds__(256) k_pairs(const uint4* __restrict__ pts, const uint32_t* __restrict__ ent,
                                               uint32_t m, G1Xyzz* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t * K >= m) return;
  r29::Xyzz acc = r29::identity();
#pragma unroll 1
  for (uint32_t e0 = t * K; e0 < t * K + K; e0 += 2 * M) {
    r29::F pre[M];
    r29::F run = r29::one();
#pragma unroll
    for (int i = 0; i < M; i++) {
      const r29::F x0 = load_x(pts, ent[e0 + 2 * i]), x1 = load_x(pts, ent[e0 + 2 * i + 1]);
      run = r29::mul(run, r29::sub<2>(x1, x0));  // prefix of dx (dx < 4p)
      pre[i] = run;
    }
    r29::F inv = INV == 0 ? inv_fermat(run) : run;
#pragma unroll
    for (int i = M - 1; i >= 0; i--) {
      r29::F x0, y0, x1, y1;
      load_xy(pts, ent[e0 + 2 * i], x0, y0);
      load_xy(pts, ent[e0 + 2 * i + 1], x1, y1);
      const r29::F dx = r29::sub<2>(x1, x0);
      const r29::F inv_i = i > 0 ? r29::mul(inv, pre[i - 1]) : inv;  // 1 / dx_i
      if (i > 0) inv = r29::mul(inv, dx);
      const r29::F lam = r29::mul(r29::sub<2>(y1, y0), inv_i);              // < 2p
      const r29::F x3 = r29::sub<2>(r29::sub<2>(r29::sqr(lam), x0), x1);   // < 6p
      const r29::F y3 = r29::sub<2>(r29::mul(lam, r29::sub<6>(x0, x3)), y0);  // < 4p
      acc = r29::madd(acc, r29::csub<1>(r29::csub<2>(r29::csub<4>(x3))), r29::csub<1>(r29::csub<2>(y3)));
    }
  }
  store_canon(acc, out + t);
}

__global__ void __launch_bounds__(256) k_inv(const uint4* __restrict__ pts, uint32_t n, G1Xyzz* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const r29::F a = load_x(pts, t);
  const r29::F r = inv_fermat(a);
  r29::to_r32(r29::mul(r, a), out[t].X.v);  // 1 (x R) when correct
}

template <typename Kern>
static float timeit(Kern k, int grid, const uint4* b, const uint32_t* ent, uint32_t m, G1Xyzz* out) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, b, ent, m, out);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 3; r++) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, b, ent, m, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

// host check: same projective point (X/ZZ, Y/ZZZ) via cross products
static size_t compare(const std::vector<G1Xyzz>& a, const std::vector<G1Xyzz>& b, size_t nt) {
  size_t bad = 0;
  for (size_t t = 0; t < nt; t++)
    if (!(a[t].X * b[t].ZZ == b[t].X * a[t].ZZ) || !(a[t].Y * b[t].ZZZ == b[t].Y * a[t].ZZZ)) bad++;
  return bad;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 24;
  const uint32_t m = 1u << lg, npts = 1u << 21;  // the 2^20-point MSM's 2^21 GLV virtual points
  // curve points (i + 1) G, i < npts, as x R' words (the library's point table form): XYZZ multiples
  // on the host, one batch inversion (Montgomery's trick) for the affine coordinates
  std::vector<uint32_t> hb(16ull * npts), he(m);
  uint64_t s = 0x243F6A8885A308D3ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
  {
    Fq one, two;
    for (int j = 0; j < 8; j++) one.v[j] = two.v[j] = 0;
    one.v[0] = 1;
    two.v[0] = 2;
    const Fq gx = fe_to_mont(one), gy = fe_to_mont(two);
    std::vector<G1Xyzz> q(npts);
    G1Xyzz acc = G1Xyzz::identity();
    for (uint32_t i = 0; i < npts; i++) q[i] = acc = xyzz_madd(acc, gx, gy);
    std::vector<Fq> pre(npts);  // prefix products of ZZZ_i
    Fq run = Fq::one();
    for (uint32_t i = 0; i < npts; i++) pre[i] = run = run * q[i].ZZZ;
    Fq inv = fe_inv(run);
    for (uint32_t i = npts; i-- > 0;) {
      const Fq izzz = i ? inv * pre[i - 1] : inv;  // 1 / ZZZ_i
      inv = inv * q[i].ZZZ;
      const Fq iz = izzz * q[i].ZZ;                // 1 / Z (ZZZ / ZZ = Z)
      const Fq x = q[i].X * (iz * iz), y = q[i].Y * izzz;
      uint32_t w[8];
      r29::to_words(r29::to_r29(x.v), w);
      for (int j = 0; j < 8; j++) hb[16ull * i + j] = w[j];
      r29::to_words(r29::to_r29(y.v), w);
      for (int j = 0; j < 8; j++) hb[16ull * i + 8 + j] = w[j];
    }
  }
  for (uint32_t e = 0; e < m; e++) he[e] = rnd() % npts;
  for (uint32_t e = 0; e + 1 < m; e += 2)  // no pair of equal points (dx = 0: not handled here)
    if (he[e + 1] == he[e]) he[e + 1] = (he[e] + 1) % npts;
  uint4* db;
  uint32_t* de;
  G1Xyzz *o1, *o2;
  const uint32_t nt = m / K;
  const int grid = (nt + 255) / 256;
  CK(hipMalloc(&db, hb.size() * 4));
  CK(hipMalloc(&de, he.size() * 4));
  CK(hipMalloc(&o1, (size_t)grid * 256 * sizeof(G1Xyzz)));
  CK(hipMalloc(&o2, (size_t)grid * 256 * sizeof(G1Xyzz)));
  CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, he.data(), he.size() * 4, hipMemcpyHostToDevice));
  std::vector<G1Xyzz> h1(nt), h2(nt);
  const float tx = timeit(k_xyzz, grid, db, de, m, o1);
  CK(hipMemcpy(h1.data(), o1, nt * sizeof(G1Xyzz), hipMemcpyDeviceToHost));
  printf("k_xyzz          %8.3f ms  %6.3f ns/entry\n", tx, tx * 1e6 / m);
  auto run = [&](auto kern, const char* name, bool check) -> int {
    const float tp = timeit(kern, grid, db, de, m, o2);
    CK(hipMemcpy(h2.data(), o2, nt * sizeof(G1Xyzz), hipMemcpyDeviceToHost));
    printf("%-15s %8.3f ms  %6.3f ns/entry  x%.3f of k_xyzz", name, tp, tp * 1e6 / m, tp / tx);
    if (check) printf("  mismatches %zu/%u", compare(h1, h2, nt), nt);
    printf("\n");
    return 0;
  };
  run(k_pairs<4, 0>, "pairs M=4 inv", true);
  run(k_pairs<8, 0>, "pairs M=8 inv", true);
  run(k_pairs<16, 0>, "pairs M=16 inv", true);
  run(k_pairs<4, 1>, "pairs M=4 noinv", false);
  run(k_pairs<8, 1>, "pairs M=8 noinv", false);
  run(k_pairs<16, 1>, "pairs M=16 noinv", false);
  {
    const uint32_t ni = m / 64;  // one inversion per lane of m / 64 lanes
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k_inv, dim3((ni + 255) / 256), dim3(256), 0, 0, db, ni, o2);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_inv, dim3((ni + 255) / 256), dim3(256), 0, 0, db, ni, o2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    std::vector<G1Xyzz> hi(1);
    CK(hipMemcpy(hi.data(), o2, sizeof(G1Xyzz), hipMemcpyDeviceToHost));
    printf("k_inv %u lanes  %8.3f ms  = %.1f XYZZ-entries of time per inversion (x R check %s)\n", ni, ms,
           ms / (tx / m) / ni, hi[0].X == Fq::one() ? "ok" : "BAD");
  }
  return 0;
}
