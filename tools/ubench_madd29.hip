// Microbenchmark (round 4): the bucket accumulation's inner step with 9 x 29-bit limbs
// (csrc/curve29.hpp madd) against the library's xyzz_madd_2p_u (8 x 32-bit, curve.hpp), in a
// k_accumulate-shaped kernel: each thread walks K consecutive entries of a random index list,
// loads the 64-byte affine point (x R words, as the library's tables), adds it into a register
// accumulator, and stores the canonical sum (x R words) at the end.  The r29 kernel converts each
// loaded point to x R' (to_r29: shift + small reduction) and the sum back (to_r32).
// Usage: ./ubench_madd29 [log2 entries = 24] [K = 64]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../snark-verifier-axiom_amd/csrc/curve.hpp"
#include "../snark-verifier-axiom_amd/csrc/curve29.hpp"

#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

using namespace sv;

__device__ __forceinline__ void load_pt(const uint4* __restrict__ b, uint32_t i, uint32_t* x, uint32_t* y) {
  const uint4 q0 = b[4 * i], q1 = b[4 * i + 1], q2 = b[4 * i + 2], q3 = b[4 * i + 3];
  x[0] = q0.x; x[1] = q0.y; x[2] = q0.z; x[3] = q0.w; x[4] = q1.x; x[5] = q1.y; x[6] = q1.z; x[7] = q1.w;
  y[0] = q2.x; y[1] = q2.y; y[2] = q2.z; y[3] = q2.w; y[4] = q3.x; y[5] = q3.y; y[6] = q3.z; y[7] = q3.w;
}

__global__ void __launch_bounds__(256) k_r32(const uint4* __restrict__ bases, const uint32_t* __restrict__ ent,
                                             uint32_t m, uint32_t K, G1Xyzz* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s0 = t * K;
  if (s0 >= m) return;
  G1Xyzz acc = G1Xyzz::identity();
  for (uint32_t e = s0; e < s0 + K && e < m; e++) {
    const uint32_t v = ent[e];
    Fq x, y;
    load_pt(bases, v & 0x7fffffffu, x.v, y.v);
    if (v & 0x80000000u) y = -y;
    acc = xyzz_madd_2p_u(acc, x, y);
  }
  out[t] = xyzz_canon2p(acc);
}

__global__ void __launch_bounds__(256) k_r29(const uint4* __restrict__ bases, const uint32_t* __restrict__ ent,
                                             uint32_t m, uint32_t K, G1Xyzz* __restrict__ out) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s0 = t * K;
  if (s0 >= m) return;
  r29::Xyzz acc = r29::identity();
  for (uint32_t e = s0; e < s0 + K && e < m; e++) {
    const uint32_t v = ent[e];
    uint32_t xw[8], yw[8];
    load_pt(bases, v & 0x7fffffffu, xw, yw);
    const r29::F x = r29::to_r29(xw);
    r29::F y = r29::to_r29(yw);
    if (v & 0x80000000u) y = r29::sub<2>(r29::zero(), y);
    acc = r29::madd(acc, x, y);
  }
  G1Xyzz r;
  r29::to_r32(acc.X, r.X.v);
  r29::to_r32(acc.Y, r.Y.v);
  r29::to_r32(acc.ZZ, r.ZZ.v);
  r29::to_r32(acc.ZZZ, r.ZZZ.v);
  out[t] = r;
}

template <typename Kern>
static float timeit(Kern k, int grid, const uint4* b, const uint32_t* ent, uint32_t m, uint32_t K, G1Xyzz* out) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, b, ent, m, K, out);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, b, ent, m, K, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
  }
  return best;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 24;
  const uint32_t K = argc > 2 ? atoi(argv[2]) : 64;
  const uint32_t m = 1u << lg, npts = 1u << 21;
  // points: random field elements below p (x R words); the addition law does not need them on the
  // curve for timing, and the two kernels' sums are compared for equality
  std::vector<uint32_t> hb(16ull * npts), he(m);
  uint64_t s = 0x243F6A8885A308D3ull;
  auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
  for (uint32_t i = 0; i < 2 * npts; i++) {
    for (int j = 0; j < 8; j++) hb[8ull * i + j] = rnd();
    hb[8ull * i + 7] &= 0x0fffffffu;  // below 2^252 < p
  }
  for (uint32_t e = 0; e < m; e++) he[e] = (rnd() % npts) | (rnd() & 0x80000000u);
  uint4* db;
  uint32_t* de;
  G1Xyzz *o32, *o29;
  const int grid = (m / K + 255) / 256;
  CK(hipMalloc(&db, hb.size() * 4));
  CK(hipMalloc(&de, he.size() * 4));
  CK(hipMalloc(&o32, (size_t)grid * 256 * sizeof(G1Xyzz)));
  CK(hipMalloc(&o29, (size_t)grid * 256 * sizeof(G1Xyzz)));
  CK(hipMemcpy(db, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(de, he.data(), he.size() * 4, hipMemcpyHostToDevice));
  const float t32 = timeit(k_r32, grid, db, de, m, K, o32);
  const float t29 = timeit(k_r29, grid, db, de, m, K, o29);
  CK(hipDeviceSynchronize());
  // the sums are the same projective points; compare affine-free: X ZZ' ... simply both canonical
  // representations of the same XYZZ point up to scaling -> compare X/ZZ and Y/ZZZ by cross products
  std::vector<G1Xyzz> h32((size_t)grid * 256), h29((size_t)grid * 256);
  CK(hipMemcpy(h32.data(), o32, h32.size() * sizeof(G1Xyzz), hipMemcpyDeviceToHost));
  CK(hipMemcpy(h29.data(), o29, h29.size() * sizeof(G1Xyzz), hipMemcpyDeviceToHost));
  size_t bad = 0, nt = m / K;
  for (size_t t = 0; t < nt; t++) {
    const G1Xyzz &a = h32[t], &b = h29[t];
    if (!(a.X * b.ZZ == b.X * a.ZZ) || !(a.Y * b.ZZZ == b.Y * a.ZZZ) || (a.ZZ.is_zero() != b.ZZ.is_zero())) bad++;
  }
  const double adds = (double)m;
  printf("entries 2^%d K %u: r32 %.3f ms (%.1f G madd/s)  r29 %.3f ms (%.1f G madd/s)  ratio %.3f  mismatches %zu/%zu\n",
         lg, K, t32, adds / t32 / 1e6, t29, adds / t29 / 1e6, t32 / t29, bad, nt);
  return bad ? 2 : 0;
}
