// Round 6 probe: the decider's w_sqr with each lane product split in two
// halves that run on DIFFERENT waves (and SIMDs) -- half A = x_lo3 y reduced by 8 word steps on
// waves 0-1, half B = x_hi5 y reduced by 5 steps on waves 2-3 (or 4-5: the same SIMDs as 0-1) --
// each half summed by its own lane_sum24, the two coefficient sums joined through LDS.  Prints
// cycles per op against wg::w_sqr and checks the results equal mod p.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_split.hip snark-verifier-axiom_amd/csrc/runtime.cpp -o tools/bin/ubench_split
#include "../snark-verifier-axiom_amd/csrc/decider.hip"

#include <cstdio>

using namespace sv;

// (a b + M p) / 2^(32 NS) with a of NA words and M < 2^(32 NS) zeroing the low NS words: product
// scanning as mont_mul, the output columns NS .. NS + 7 (the value is below 2^256 for the two
// shapes used here: NA = 3, NS = 8 below 2^95 + p; NA = 5, NS = 5 below 2^255 + p)
template <int NA, int NS>
__device__ __forceinline__ Fq mont_part(const uint32_t* a, const Fq& b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return b;  // (device-only: the mac helpers are device asm)
#else
  uint32_t m[NS], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < NS + 8; k++) {
    uint32_t xs[16], ys[16];
    int c = 0;
#pragma unroll
    for (int i = 0; i < NA; i++) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        xs[c] = a[i];
        ys[c] = b.v[j];
        c++;
      }
    }
#pragma unroll
    for (int i = 0; i < NS; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 8) {
        xs[c] = m[i];
        ys[c] = FqTag::p(j);
        c++;
      }
    }
    int q = 0;
    bool open = false;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
      open = true;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
      open = true;
    } else if (c == 1) {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
      open = true;
    }
#pragma unroll
    for (; q + 3 < c; q += 4) mac_carry4(acc, ovf, xs + q, ys + q);
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    if (k < NS) {
      m[k] = (uint32_t)acc * FqTag::NP0;
      if (open) mac_carry(acc, ovf, m[k], FqTag::p(0));
      else mac_first(acc, ovf, m[k], FqTag::p(0));
    } else {
      t[k - NS] = (uint32_t)acc;
      if (!open) ovf = 0;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  Fq r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = t[j];
  return r;
#endif
}

// Round 6, in-wave split: lane t of waves 0-2 computes HALF of virtual lane u = 32 (t >> 6) + (t & 31)'s
// product -- lanes 0-31 of a wave the low words x_lo of x, lanes 32-63 the high words x_hi -- in ONE
// instruction stream: 16 product-scanning columns of the 4 x 8 product, the reduction factor m_k of
// columns k >= 4 zeroed on the hi lanes, so they divide by 2^128 and the lo lanes by 2^256:
//   lo: (x_lo y + M p) / 2^256 < p + 1,  hi: (x_hi y + M' p) / 2^128 < 2p   (x, y < 2p)
// and lo + hi = (x_lo + 2^128 x_hi) y / 2^256 = x y / 2^256 (mod p), below 3p.
__device__ __forceinline__ Fq mont_half(const uint32_t* a, const Fq& b, bool hi) {
#if !defined(__HIP_DEVICE_COMPILE__)
  (void)a; (void)hi;
  return b;
#else
  uint32_t m[8], t[8], w[4];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    uint32_t xs[16], ys[16];
    int c = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        xs[c] = a[i];
        ys[c] = b.v[j];
        c++;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 8) {
        xs[c] = m[i];
        ys[c] = FqTag::p(j);
        c++;
      }
    }
    int q = 0;
    bool open = false;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
      open = true;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
      open = true;
    } else if (c == 1) {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
      open = true;
    }
#pragma unroll
    for (; q + 3 < c; q += 4) mac_carry4(acc, ovf, xs + q, ys + q);
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    if (k < 8) {
      m[k] = (uint32_t)acc * FqTag::NP0;
      if (k >= 4 && hi) m[k] = 0;
      if (open) mac_carry(acc, ovf, m[k], FqTag::p(0));
      else mac_first(acc, ovf, m[k], FqTag::p(0));
      if (k >= 4) w[k - 4] = (uint32_t)acc;
    } else {
      t[k - 8] = (uint32_t)acc;
      if (!open) ovf = 0;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  Fq r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = hi ? (j < 4 ? w[j] : t[j - 4]) : t[j];
  return r;
#endif
}

// w_sqr over the in-wave split (V: the roles of virtual lane u; lanes 0-31 of waves 0-2 store)
__device__ __forceinline__ void w_sqr_inwave(const wg::WLane& V, Fq2* __restrict__ dst, const Fq2* a) {
  using namespace wg;
  const int t = threadIdx.x;
  if (t < 192) {
    const bool hi = (t & 32) != 0;
    const int q = V.sq;
    const bool square = V.ssquare;
    const bool xc1 = square ? q == 1 : (q & 1);
    const bool yc1 = square ? q != 0 : (q == 1 || q == 2);
    const Fq x = ld_fq(xc1 ? &a[V.si].c1 : &a[V.si].c0);
    const Fq y = ld_fq(yc1 ? &a[V.sj].c1 : &a[V.sj].c0);
    uint32_t xh[4];
#pragma unroll
    for (int k = 0; k < 4; k++) xh[k] = hi ? x.v[4 + k] : x.v[k];
    const Fq h = mont_half(xh, y, hi);
    Fq v;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t o = (uint32_t)__builtin_amdgcn_permlane32_swap((int)h.v[k], (int)h.v[k], false, false)[1];
      v.v[k] = __builtin_addc(h.v[k], o, c, &c);
    }
    const Lz s = lane_sum24<4>(v, V.skeep, V.ssend);
    if (!hi && V.sgrp) store_coeff(dst, V.sk, t & 15, s);
  }
  __syncthreads();
}

// w_sqr with split lane products: lanes t < 128 half A, lanes [OFF, OFF + 128) half B for lane
// t - OFF (OFF = 128: waves 2-3, other SIMDs; OFF = 256: waves 4-5, the same SIMDs as 0-1);
// xch: 6 coefficients x 2 (re, im) Lz values
template <int OFF>
__device__ __forceinline__ void w_sqr_split(const wg::WLane& L, const wg::WLane& LB, Fq2* __restrict__ dst,
                                            const Fq2* a, wg::Lz* xch) {
  using namespace wg;
  const int t = threadIdx.x;
  const bool ha = t < 128, hb = t >= OFF && t < OFF + 128;
  if (ha || hb) {
    const WLane& M = ha ? L : LB;  // (wave-uniform choice)
    const int q = M.sq;
    const bool square = M.ssquare;
    const bool xc1 = square ? q == 1 : (q & 1);
    const bool yc1 = square ? q != 0 : (q == 1 || q == 2);
    const Fq x = ld_fq(xc1 ? &a[M.si].c1 : &a[M.si].c0);
    const Fq y = ld_fq(yc1 ? &a[M.sj].c1 : &a[M.sj].c0);
    Fq v;
    if (ha) v = mont_part<3, 8>(x.v, y);
    else v = mont_part<5, 5>(x.v + 3, y);
    const Lz s = lane_sum24<4>(v, M.skeep, M.ssend);
    const int j = t & 15;
    if (hb && M.sgrp && j < 2) xch[M.sk * 2 + j] = s;
    __syncthreads();
    if (ha && M.sgrp && j < 2) {
      const Lz o = xch[M.sk * 2 + j];
      st_fq(j ? &dst[M.sk].c1 : &dst[M.sk].c0, lz_reduce(lz_add(s, o)));
    }
  } else {
    __syncthreads();
  }
  __syncthreads();
}

// the WLane of lane t - off (the B half's roles)
__device__ wg::WLane wlane_of(int off) {
  // wlane_init reads threadIdx.x: recompute the square fields for t - off by hand
  wg::WLane L = wg::wlane_init();
  const int t = (int)threadIdx.x - off;
  if (t >= 0 && t < 128) {
    const int grp = t >> 4, j = t & 15;
    L.sgrp = grp < 6;
    L.sk = L.sgrp ? grp : 0;
    L.sq = j & 3;
    const SqrTerm tm = c_sqr[L.sk][j >> 2];
    L.slive = L.sgrp && tm.i >= 0;
    L.si = L.slive ? tm.i : 0;
    L.sj = L.slive ? tm.j : 0;
    L.ssquare = L.si == L.sj;
    L.sxi = L.slive && tm.xi;
    const int q = L.sq, f = L.ssquare ? 1 : 2;
    int re = q == 0 ? f : (q == 1 ? -f : 0), im = q == 2 ? 2 : (q == 3 && !L.ssquare ? 2 : 0);
    if (!L.slive) re = im = 0;
    wg::keep_send(re, im, L.sxi, L.skeep, L.ssend);
  }
  return L;
}

// the w_sqr roles of virtual lane u = 32 (t >> 6) + (t & 31) (same parity as t)
__device__ wg::WLane wlane_virt() {
  wg::WLane L = wg::wlane_init();
  const int t = threadIdx.x, u = 32 * (t >> 6) + (t & 31);
  const int grp = u >> 4, j = u & 15;
  L.sgrp = grp < 6;
  L.sk = L.sgrp ? grp : 0;
  L.sq = j & 3;
  const SqrTerm tm = c_sqr[L.sk][j >> 2];
  L.slive = L.sgrp && tm.i >= 0;
  L.si = L.slive ? tm.i : 0;
  L.sj = L.slive ? tm.j : 0;
  L.ssquare = L.si == L.sj;
  L.sxi = L.slive && tm.xi;
  const int q = L.sq, f = L.ssquare ? 1 : 2;
  int re = q == 0 ? f : (q == 1 ? -f : 0), im = q == 2 ? 2 : (q == 3 && !L.ssquare ? 2 : 0);
  if (!L.slive) re = im = 0;
  wg::keep_send(re, im, L.sxi, L.skeep, L.ssend);
  return L;
}

// mode 0: wg::w_sqr; 1: split with B on waves 2-3; 2: split with B on waves 4-5 (512 threads);
// 3: the in-wave split (waves 0-2)
template <int MODE>
__global__ void __launch_bounds__(512) k_op(int iters, unsigned long long* cycles, uint32_t* out) {
  __shared__ Fq2 S[2 * 6];
  __shared__ wg::Lz xch[12];
  const int t = threadIdx.x;
  if (t < 6) {
    S[t] = Fq2::one();
    S[t].c1 = Fq::one();
    S[t].c0.v[0] ^= 0x12345u * (t + 1);
    S[t].c1.v[1] ^= 0x777u * (t + 3);
  }
  __syncthreads();
  Fq2* a = S;
  Fq2* c = S + 6;
  const wg::WLane L = wg::wlane_init();
  const wg::WLane LB = MODE == 3 ? wlane_virt() : wlane_of(MODE == 2 ? 256 : 128);
  const unsigned long long t0 = clock64();
  for (int i = 0; i < iters; i++) {
    if constexpr (MODE == 0) wg::w_sqr(L, c, a);
    else if constexpr (MODE == 3) w_sqr_inwave(LB, c, a);
    else w_sqr_split<MODE == 1 ? 128 : 256>(L, LB, c, a, xch);
    Fq2* tmp = a;
    a = c;
    c = tmp;
  }
  const unsigned long long t1 = clock64();
  if (t == 0) *cycles = t1 - t0;
  if (t < 12) {  // canonical coefficients
    const Fq v = wg::fq_canon((t & 1) ? a[t >> 1].c1 : a[t >> 1].c0);
    for (int k = 0; k < 8; k++) out[8 * t + k] = v.v[k];
  }
}

int main() {
  unsigned long long* dc;
  uint32_t* dout;
  (void)hipMalloc(&dc, 8);
  (void)hipMalloc(&dout, 4 * 96 * 4);
  const char* names[] = {"w_sqr", "split B@waves2-3", "split B@waves4-5", "in-wave split"};
  void (*ks[4])(int, unsigned long long*, uint32_t*) = {k_op<0>, k_op<1>, k_op<2>, k_op<3>};
  uint32_t h[4][96];
  for (int threads : {256, 512}) {
    for (int m = 0; m < 4; m++) {
      if (m == 2 && threads == 256) continue;
      for (int iters : {7, 207}) {
        hipLaunchKernelGGL(ks[m], dim3(1), dim3(threads), 0, 0, iters, dc, dout + 96 * m);
        unsigned long long c = 0;
        (void)hipMemcpy(&c, dc, 8, hipMemcpyDeviceToHost);
        if (iters == 207) printf("%4d threads %-18s %8.1f cycles/op\n", threads, names[m], (double)c / iters);
      }
    }
    (void)hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
    bool same = true;
    for (int m = 1; m < 4; m++)
      for (int k = 0; k < 96; k++)
        if (!(m == 2 && threads == 256) && h[m][k] != h[0][k]) same = false;
    printf("%4d threads: results equal mod p: %s\n", threads, same ? "yes" : "NO");
  }
  return 0;
}
