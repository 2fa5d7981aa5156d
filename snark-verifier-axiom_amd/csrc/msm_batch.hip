// f1: many small MSMs in ONE launch: the per-proof MSMs of native
// verification (bdfg21.rs:75-78, gwc19.rs:76-79 via Msm::evaluate -> NativeLoader::
// multi_scalar_multiplication, native.rs:61-71) and the two accumulation MSMs of
// KzgAs::create_proof (accumulation.rs:177-192) are tens to thousands of terms each -- far too
// small to fill 256 CUs one at a time (the single-MSM pipeline is launch/latency bound there).
//
// One workgroup (256 threads) per MSM, everything in LDS, signed c-bit windows (c = 5 for small
// batches, 8 for larger MSMs):
//   1. chunk of NCH terms: scalars -> W signed digits (LDS), LDS-atomic histogram per (window,
//      bucket), per-window exclusive scan, scatter of term indices into per-bucket lists;
//   2. G = min(2^(c-1), 64) lanes per window: each lane sums its buckets' lists with mixed XYZZ
//      adds, weights them by the bucket magnitude (short double-and-add), and the G lanes fold
//      with xor-shuffles; the group leader adds the window sum into T[w] (LDS, kept across chunks);
//   3. one wave per MSM: Horner over the windows (~255 doublings), the independent products of
//      each doubling / addition spread over 4 lanes (3-4 product levels instead of 9-14), then
//      one binary-EEA inversion, affine out.
// Steps 1-2 run as (MSM, window group) blocks so even one MSM spreads over several CUs; step 3
// is a dependent chain per MSM (one wave each), so a batch costs about one chain whatever its
// size.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "curve.hpp"
#include "glv.hpp"
#include "host_ec.hpp"
#include "msm_batch.hpp"
#include "quad.hpp"
#include "runtime.hpp"

namespace sv {

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ Fq ld_fq(const uint32_t* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  Fq r;
  r.v[0] = a.x, r.v[1] = a.y, r.v[2] = a.z, r.v[3] = a.w;
  r.v[4] = b.x, r.v[5] = b.y, r.v[6] = b.z, r.v[7] = b.w;
  return r;
}

__device__ __forceinline__ void st_fq(uint32_t* p, const Fq& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  q[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}

__device__ __forceinline__ Fq shfl_xor_fq(const Fq& a, int m) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)__shfl_xor((int)a.v[i], m);
  return r;
}

__device__ __forceinline__ G1Xyzz shfl_xor_pt(const G1Xyzz& p, int m) {
  return {shfl_xor_fq(p.X, m), shfl_xor_fq(p.Y, m), shfl_xor_fq(p.ZZ, m), shfl_xor_fq(p.ZZZ, m)};
}

// k * P for 1 <= k <= 128, MSB first
__device__ __forceinline__ G1Xyzz smul_small(const G1Xyzz& p, uint32_t k) {
  G1Xyzz r = p;
  const int top = 31 - __clz(k);
  for (int b = top - 1; b >= 0; b--) {
    r = xyzz_dbl(r);
    if ((k >> b) & 1) r = xyzz_add(r, p);
  }
  return r;
}

// GLV (glv.hpp): every term k P is split into k1 P + k2 phi(P) with |k_i| < 2^127, so the windows
// cover 128 bits and the per-MSM Horner chain is ~128 doublings instead of ~255.
template <int C>
struct BatchCfg {
  static constexpr int W = (128 + C - 1) / C;  // signed digits of a < 2^127 half scalar
  static constexpr int B = 1 << (C - 1);
  static constexpr int G = B < 64 ? B : 64;  // lanes per window
  static constexpr int BPL = B / G;          // buckets per lane
  static constexpr int WPB = kThreads / G;   // windows per block
  static constexpr int WG = (W + WPB - 1) / WPB;  // window groups (blockIdx.y)
  static constexpr int NCH = C <= 6 ? 128 : 256;
};

// Step 1 + 2: block (msm, window group) -> window sums Tg[id * W + w] (XYZZ, Montgomery).
template <int C>
__global__ void __launch_bounds__(kThreads) k_msm_batch_windows(const G1Aff* __restrict__ bases,
                                                                 const Fr* __restrict__ scalars,
                                                                 const uint64_t* __restrict__ off,
                                                                 const uint32_t* __restrict__ ids, int mont,
                                                                 G1Xyzz* __restrict__ Tg, uint32_t* __restrict__ err,
                                                                 const uint32_t* __restrict__ bidx, uint64_t tlen,
                                                                 int mont_b) {
  using Cf = BatchCfg<C>;
  constexpr int W = Cf::W, B = Cf::B, G = Cf::G, BPL = Cf::BPL, WPB = Cf::WPB, NCH = Cf::NCH;
  __shared__ uint32_t cur[WPB * B];       // histogram, then scatter cursors (= bucket ends)
  __shared__ uint16_t bst[WPB * B];       // bucket starts within the window's list
  __shared__ uint16_t dig[2 * NCH * WPB]; // magnitude | sign << 8, per (half term, window)
  __shared__ uint16_t lst[WPB * 2 * NCH]; // half-term index (term | half << 8) | sign << 15
  __shared__ G1Xyzz T[WPB];               // window sums of this block's windows

  const int tid = threadIdx.x;
  const uint32_t id = ids ? ids[blockIdx.x] : blockIdx.x;  // optional indirection (host API skips big MSMs)
  const int w0 = blockIdx.y * WPB;
  const int nw = W - w0 < WPB ? W - w0 : WPB;
  const uint64_t b0 = off[id], e0 = off[id + 1];
  if (tid < WPB) T[tid] = G1Xyzz::identity();
  const Fq beta = fq_const(GLV_BETA_MONT);

  for (uint64_t c0 = b0; c0 < e0; c0 += NCH) {
    const int m = (int)(e0 - c0 < (uint64_t)NCH ? e0 - c0 : (uint64_t)NCH);
    for (int i = tid; i < WPB * B; i += kThreads) cur[i] = 0;
    __syncthreads();
    if (tid < m) {
      Fr s;
      {
        const Fq t = ld_fq(reinterpret_cast<const uint32_t*>(scalars + c0 + tid));
#pragma unroll
        for (int i = 0; i < 8; i++) s.v[i] = t.v[i];
      }
      if (!s.is_reduced()) atomicOr(err, 2u);
      if (mont) s = fe_from_mont(s);
      uint32_t hv[2][4];
      glv_split(s.v, hv[0], hv[1]);
      for (int h = 0; h < 2; h++) {
        const uint32_t sg = hv[h][3] >> 31;
        hv[h][3] &= 0x7fffffffu;
        // signed digits: the carry runs from window 0, only this block's windows are kept
        uint32_t carry = 0;
        for (int w = 0; w < w0 + nw; w++) {
          const int pos = w * C, limb = pos >> 5, sh = pos & 31;
          const uint32_t lo = limb < 4 ? hv[h][limb] : 0u;
          const uint32_t hi = limb + 1 < 4 ? hv[h][limb + 1] : 0u;
          uint32_t bits = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
          bits = (bits & ((1u << C) - 1)) + carry;
          uint32_t mag, neg;
          if (bits > (uint32_t)B) {  // digit bits - 2^C < 0 (bits == 2^C: digit 0, carry 1)
            mag = (1u << C) - bits;
            neg = mag ? 1u : 0u;
            carry = 1;
          } else {
            mag = bits;
            neg = 0;
            carry = 0;
          }
          if (w >= w0) {
            const int lw = w - w0;
            dig[(h * NCH + tid) * WPB + lw] = (uint16_t)(mag | ((neg ^ sg) << 8));
            if (mag) atomicAdd(&cur[lw * B + mag - 1], 1u);
          }
        }
      }
    }
    __syncthreads();
    if (tid < nw) {
      uint32_t acc = 0;
      for (int b = 0; b < B; b++) {
        const uint32_t c = cur[tid * B + b];
        bst[tid * B + b] = (uint16_t)acc;
        cur[tid * B + b] = acc;
        acc += c;
      }
    }
    __syncthreads();
    if (tid < m) {
      for (int h = 0; h < 2; h++)
        for (int lw = 0; lw < nw; lw++) {
          const uint32_t d = dig[(h * NCH + tid) * WPB + lw];
          const uint32_t mag = d & 0xff;
          if (mag) {
            const uint32_t pos = atomicAdd(&cur[lw * B + mag - 1], 1u);
            lst[lw * 2 * NCH + pos] = (uint16_t)(tid | (h << 8) | ((d >> 8) << 15));
          }
        }
    }
    __syncthreads();
    {
      const int lw = tid / G;
      const int g = tid % G;
      G1Xyzz part = G1Xyzz::identity();
      if (lw < nw) {
        for (int k = 0; k < BPL; k++) {
          const int b = g + k * G;  // magnitude b + 1
          G1Xyzz acc = G1Xyzz::identity();
          const uint32_t pe = cur[lw * B + b];
          for (uint32_t p = bst[lw * B + b]; p < pe; p++) {
            const uint32_t e = lst[lw * 2 * NCH + p];
            uint64_t bi = c0 + (e & 0xff);
            if (bidx) {  // base table: term -> table row (fixed bases resident on the device)
              const uint32_t ti = bidx[bi];
              if (ti >= tlen) {
                atomicOr(err, 4u);
                continue;
              }
              bi = ti;
            }
            const uint32_t* bp = reinterpret_cast<const uint32_t*>(bases + bi);
            Fq x = ld_fq(bp), y = ld_fq(bp + 8);
            if (!x.is_reduced() || !y.is_reduced()) {  // same contract as the single-MSM path
              atomicOr(err, 1u);
              continue;
            }
            if (x.is_zero() && y.is_zero()) continue;  // identity base
            if (!mont_b) {
              x = fe_to_mont(x);
              y = fe_to_mont(y);
            }
            if ((e >> 8) & 1) x = x * beta;  // phi(P) = (beta x, y)
            if (e >> 15) y = -y;
            acc = xyzz_madd_2p(acc, x, y);  // 2p domain (curve.hpp), canonical before smul_small
          }
          if (!acc.is_identity()) part = xyzz_add(part, smul_small(xyzz_canon2p(acc), (uint32_t)b + 1));
        }
      }
#pragma unroll
      for (int s = 1; s < G; s <<= 1) part = xyzz_add(part, shfl_xor_pt(part, s));
      if (g == 0 && lw < nw) T[lw] = xyzz_add(T[lw], part);
    }
    __syncthreads();
  }
  if (tid < nw) Tg[(size_t)blockIdx.x * W + w0 + tid] = T[tid];  // by batch position (ids may skip MSMs)
}

// ---- Steps 1 + 2, quad form (default for c = 5, i.e. MSMs of <= 256 terms) ----------------------
// k_batch_prep: one thread per term, once: scalar checks + GLV split + the signed digits of every
// window of both halves (u8: magnitude | sign << 7, laid out [msm][window][half-term] so a window's
// wave reads them contiguously), and the term's two points P and phi(P) = (beta x, y) in Montgomery
// form (bases checked / converted / looked up in the table here, identity (0, 0) kept).
// k_batch_windows_q: one wave per (MSM, window): an LDS counting sort of the window's digits into its
// B = 16 buckets, then ONE QUAD of lanes per bucket summing its entries with quad-form mixed adds
// (quad.hpp), then sum_b (b + 1) S_b = sum_b R_b over the suffix sums R_b = sum_{b' >= b} S_b': a
// 4-level scan and a 4-level tree across the wave's 16 quads.  The old kernel ran ~20 dependent
// whole additions per window on one wave per SIMD (a per-lane bucket chain, a divergent weighting
// double-and-add, a shuffle tree); here every level is one quad operation.
constexpr int kQC = 5;                       // window bits of the quad path
constexpr int kQB = 1 << (kQC - 1);          // 16 buckets: one quad each in a 64-lane wave
constexpr int kQW = BatchCfg<kQC>::W;        // 26 windows of a 128-bit GLV half
constexpr int kQMaxTerms = 256;              // half-terms of one window sorted in LDS at once

__global__ void __launch_bounds__(kThreads) k_batch_prep(const G1Aff* __restrict__ bases,
                                                         const Fr* __restrict__ scalars,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ ids, int mont,
                                                         uint32_t max_terms, uint8_t* __restrict__ dig,
                                                         G1Aff* __restrict__ pts, uint32_t* __restrict__ err,
                                                         const uint32_t* __restrict__ bidx, uint64_t tlen,
                                                         int mont_b) {
  const uint32_t k = blockIdx.x;  // position in the batch
  const uint32_t id = ids ? ids[k] : k;
  const uint64_t b0 = off[id], e0 = off[id + 1];
  const uint32_t i = blockIdx.y * kThreads + threadIdx.x;  // term of this MSM
  if (b0 + i >= e0) return;
  const uint64_t t = b0 + i;
  Fr s;
  {
    const Fq q = ld_fq(reinterpret_cast<const uint32_t*>(scalars + t));
#pragma unroll
    for (int j = 0; j < 8; j++) s.v[j] = q.v[j];
  }
  if (!s.is_reduced()) atomicOr(err, 2u);
  if (mont) s = fe_from_mont(s);
  uint64_t bi = t;
  if (bidx) {
    const uint32_t ti = bidx[t];
    if (ti >= tlen) {
      atomicOr(err, 4u);
      s = Fr::zero();
      bi = 0;
    } else {
      bi = ti;
    }
  }
  uint32_t hv[2][4];
  glv_split(s.v, hv[0], hv[1]);
  const size_t HM = 2 * (size_t)max_terms;  // half-terms per (msm, window) row
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const uint32_t sg = hv[h][3] >> 31;
    hv[h][3] &= 0x7fffffffu;
    uint32_t carry = 0;
    for (int w = 0; w < kQW; w++) {
      const int pos = w * kQC, limb = pos >> 5, sh = pos & 31;
      const uint32_t lo = limb < 4 ? hv[h][limb] : 0u;
      const uint32_t hi = limb + 1 < 4 ? hv[h][limb + 1] : 0u;
      uint32_t bits = sh ? ((lo >> sh) | (hi << (32 - sh))) : lo;
      bits = (bits & ((1u << kQC) - 1)) + carry;
      uint32_t mag, neg;
      if (bits > (uint32_t)kQB) {  // digit bits - 2^C < 0 (bits == 2^C: digit 0, carry 1)
        mag = (1u << kQC) - bits;
        neg = mag ? 1u : 0u;
        carry = 1;
      } else {
        mag = bits;
        neg = 0;
        carry = 0;
      }
      dig[((size_t)k * kQW + w) * HM + 2 * i + h] = (uint8_t)(mag | ((neg ^ sg) << 7));
    }
  }
  const uint32_t* bp = reinterpret_cast<const uint32_t*>(bases + bi);
  Fq x = ld_fq(bp), y = ld_fq(bp + 8);
  if (!x.is_reduced() || !y.is_reduced()) {  // same contract as the single-MSM path
    atomicOr(err, 1u);
    x = y = Fq::zero();
  }
  const bool ident = x.is_zero() && y.is_zero();
  if (!mont_b && !ident) {
    x = fe_to_mont(x);
    y = fe_to_mont(y);
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(pts + 2 * ((size_t)k * max_terms + i));
  st_fq(o, x);
  st_fq(o + 8, y);
  st_fq(o + 16, x * fq_const(GLV_BETA_MONT));  // phi(P); the identity maps to itself
  st_fq(o + 24, y);
}

// acc (quad form, 2p domain) + the affine point (x2, y2) (reduced, not the identity): madd-2008-s
// in 4 levels -- U2 = x2 ZZ1 | S2 = y2 ZZZ1, then PP = P^2 | RR = R^2, then PPP | Q = X1 PP |
// ZZ3 = ZZ1 PP, then R (Q - X3) | Y1 PPP | ZZZ3 = ZZZ1 PPP
__device__ __forceinline__ Fq quad_madd_2p(const Fq& a, const Fq& x2, const Fq& y2, int c) {
  using namespace quad;
  const Fq zz = perm<qp(2, 2, 2, 2)>(a), zzz = perm<qp(3, 3, 3, 3)>(a);
  const Fq X1 = perm<qp(0, 0, 0, 0)>(a), Y1 = perm<qp(1, 1, 1, 1)>(a);
  const Fq L1 = fe_mul_lazy(c == 0 ? x2 : y2, c == 0 ? zz : zzz);  // q0 U2, q1 S2 (q2, q3 repeat q1)
  const Fq d = fe_sub2p(perm<qp(0, 1, 1, 1)>(L1), pick(c == 0, X1, Y1));  // q0 P, q1..3 R
  const Fq L2 = fe_mul_lazy(d, d);                                       // q0 PP, q1 RR
  const Fq PP = perm<qp(0, 0, 0, 0)>(L2), P = perm<qp(0, 0, 0, 0)>(d);
  const Fq L3 = fe_mul_lazy(c == 0 ? P : (c == 1 ? X1 : zz), PP);        // q0 PPP, q1 Q, q2 ZZ3
  const Fq PPP = perm<qp(0, 0, 0, 0)>(L3), Q = perm<qp(1, 1, 1, 1)>(L3);
  const Fq X3 = fe_sub2p(fe_sub2p(fe_sub2p(perm<qp(1, 1, 1, 1)>(L2), PPP), Q), Q);
  const Fq R = perm<qp(1, 1, 1, 1)>(d);
  const Fq L4 = fe_mul_lazy(c == 0 ? R : (c == 1 ? Y1 : zzz), c == 0 ? fe_sub2p(Q, X3) : PPP);
  const Fq Y3 = fe_sub2p(perm<qp(0, 0, 0, 0)>(L4), perm<qp(1, 1, 1, 1)>(L4));
  // the lane moves run on every lane of the quad BEFORE the per-lane choice: a DPP move inside a
  // ?: branch executes with the other lanes masked off and reads a dead source lane
  const Fq ZZ3 = perm<qp(2, 2, 2, 2)>(L3), ZZZ3 = perm<qp(2, 2, 2, 2)>(L4);
  Fq r = c == 0 ? X3 : (c == 1 ? Y3 : (c == 2 ? ZZ3 : ZZZ3));
  const bool a_id = zz.is_zero();
  const bool p0 = fe_is_zero2p(P), r0 = fe_is_zero2p(R);
  const bool same = !a_id && p0 && r0;
  if (__builtin_expect(__any(same), 0)) {
    const Fq t = dbl_2p_cold(a, c);
    if (same) r = t;
  }
  if (!a_id && p0 && !r0) r = Fq::zero();
  if (a_id) r = c == 0 ? x2 : (c == 1 ? y2 : Fq::one());  // (x2, y2, 1, 1)
  return r;
}

__global__ void __launch_bounds__(64) k_batch_windows_q(const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ ids, uint32_t max_terms,
                                                        const uint8_t* __restrict__ dig,
                                                        const G1Aff* __restrict__ pts, G1Xyzz* __restrict__ Tg) {
  __shared__ uint32_t cnt[kQB], start[kQB + 1];
  __shared__ uint16_t lst[2 * kQMaxTerms];
  const uint32_t k = blockIdx.x, w = blockIdx.y, lane = threadIdx.x;
  const uint32_t id = ids ? ids[k] : k;
  const uint32_t m = (uint32_t)(off[id + 1] - off[id]);
  const uint8_t* dg = dig + ((size_t)k * kQW + w) * 2 * (size_t)max_terms;
  if (lane < kQB) cnt[lane] = 0;
  __syncthreads();
  for (uint32_t j = lane; j < 2 * m; j += 64) {
    const uint32_t d = dg[j];
    if (d & 0x7f) atomicAdd(&cnt[(d & 0x7f) - 1], 1u);
  }
  __syncthreads();
  if (lane == 0) {
    uint32_t a = 0;
    for (int b = 0; b < kQB; b++) {
      start[b] = a;
      a += cnt[b];
      cnt[b] = start[b];
    }
    start[kQB] = a;
  }
  __syncthreads();
  for (uint32_t j = lane; j < 2 * m; j += 64) {
    const uint32_t d = dg[j];
    if (d & 0x7f) lst[atomicAdd(&cnt[(d & 0x7f) - 1], 1u)] = (uint16_t)(j | ((d >> 7) << 15));
  }
  __syncthreads();
  // quad b sums bucket b (digit magnitude b + 1); every branch is uniform within the quad
  const int c = lane & 3, b = lane >> 2;
  const G1Aff* pk = pts + 2 * (size_t)k * max_terms;
  Fq S = Fq::zero();
  for (uint32_t e = start[b]; e < start[b + 1]; e++) {
    const uint32_t v = lst[e];
    const uint32_t* pp = reinterpret_cast<const uint32_t*>(pk + (v & 0x7fff));
    const Fq x = ld_fq(pp);
    Fq y = ld_fq(pp + 8);
    if (x.is_zero() && y.is_zero()) continue;  // identity base
    if (v >> 15) y = -y;
    S = quad_madd_2p(S, x, y, c);
  }
  // suffix sums R_b = sum_{b' >= b} S_b' (Hillis-Steele over the quads), then sum_b R_b (unrolled:
  // rolled loops with run-time shuffle distances measured slower, 525 -> 642 us for 128 x 64)
#pragma unroll
  for (int dq = 1; dq < kQB; dq <<= 1) {
    const Fq o = quad::down(S, 4 * dq);
    if (b + dq < kQB) S = quad::add_2p(S, o, c);
  }
#pragma unroll
  for (int dq = kQB / 2; dq >= 1; dq >>= 1) {
    const Fq o = quad::down(S, 4 * dq);
    if (b < dq) S = quad::add_2p(S, o, c);
  }
  if (b == 0) quad::st(Tg + (size_t)k * kQW + w, c, fe_canon2p(S));
}

// ---- Steps 2 + 3, bucket-wise Horner (default for c = 5): sum_w 2^(5w) sum_b (b+1) S_wb is
// regrouped as sum_b (b+1) H_b with H_b = sum_w 2^(5w) S_wb, so the bucket weighting (a 4-level scan
// and a 4-level tree of quad additions) runs ONCE per MSM after the Horner instead of once per
// window, and the window kernel only sums buckets.  The Horner then runs 16 chains per MSM (one quad
// per bucket, one wave per MSM) instead of one: the same dependent depth, and the extra work lands
// on SIMDs the single chain left idle.
// bucket_window: one wave per (MSM, window): the LDS counting sort of k_batch_windows_q, then lane
// 4b + j sums every 4th entry of bucket b from the j-th with scalar 2p-domain mixed adds (a chain of
// ~2 adds, ~4 at most: no quad overhead while the quad's lanes hold independent work), the quad's
// four partial sums go to quad form (quad::transpose) and are added in two levels.
struct BucketSmem {
  uint32_t cnt[kQB], start[kQB + 1];
  uint16_t lst[2 * kQMaxTerms];
};

// lane 4b + c of the wave returns the sum of every 4th entry of bucket b (from the c-th) of window w
// of batch entry k: the LDS counting sort of the window's digits, then a chain of mixed additions
__device__ __forceinline__ G1Xyzz bucket_chain(BucketSmem& sm, uint32_t k, uint32_t w, const uint64_t* __restrict__ off,
                                           const uint32_t* __restrict__ ids, uint32_t max_terms,
                                           const uint8_t* __restrict__ dig, const G1Aff* __restrict__ pts) {
  const uint32_t lane = threadIdx.x;
  const uint32_t id = ids ? ids[k] : k;
  const uint32_t m = (uint32_t)(off[id + 1] - off[id]);
  const uint8_t* dg = dig + ((size_t)k * kQW + w) * 2 * (size_t)max_terms;
  if (lane < kQB) sm.cnt[lane] = 0;
  __syncthreads();
  for (uint32_t j = lane; j < 2 * m; j += 64) {
    const uint32_t d = dg[j];
    if (d & 0x7f) atomicAdd(&sm.cnt[(d & 0x7f) - 1], 1u);
  }
  __syncthreads();
  if (lane == 0) {
    uint32_t a = 0;
    for (int b = 0; b < kQB; b++) {
      sm.start[b] = a;
      a += sm.cnt[b];
      sm.cnt[b] = sm.start[b];
    }
    sm.start[kQB] = a;
  }
  __syncthreads();
  for (uint32_t j = lane; j < 2 * m; j += 64) {
    const uint32_t d = dg[j];
    if (d & 0x7f) sm.lst[atomicAdd(&sm.cnt[(d & 0x7f) - 1], 1u)] = (uint16_t)(j | ((d >> 7) << 15));
  }
  __syncthreads();
  const int c = lane & 3, b = lane >> 2;
  const G1Aff* pk = pts + 2 * (size_t)k * max_terms;
  G1Xyzz acc = G1Xyzz::identity();
  for (uint32_t e = sm.start[b] + c; e < sm.start[b + 1]; e += 4) {
    const uint32_t v = sm.lst[e];
    const uint32_t* pp = reinterpret_cast<const uint32_t*>(pk + (v & 0x7fff));
    const Fq x = ld_fq(pp);
    Fq y = ld_fq(pp + 8);
    if (x.is_zero() && y.is_zero()) continue;  // identity base
    if (v >> 15) y = -y;
    acc = xyzz_madd_2p(acc, x, y);
  }
  return acc;
}

// quad b of the wave returns S_b (quad form, 2p domain) of window w of batch entry k
__device__ __forceinline__ Fq bucket_sum_q(BucketSmem& sm, uint32_t k, uint32_t w, const uint64_t* __restrict__ off,
                                           const uint32_t* __restrict__ ids, uint32_t max_terms,
                                           const uint8_t* __restrict__ dig, const G1Aff* __restrict__ pts) {
  const G1Xyzz acc = bucket_chain(sm, k, w, off, ids, max_terms, dig, pts);
  const int c = threadIdx.x & 3;
  Fq q[4] = {acc.X, acc.Y, acc.ZZ, acc.ZZZ};
  quad::transpose(q, c);  // lane c: coordinate c of the quad's four partial sums
  const Fq s01 = quad::add_2p(q[0], q[1], c), s23 = quad::add_2p(q[2], q[3], c);
  return quad::add_2p(s01, s23, c);
}

__device__ __forceinline__ void bucket_window(BucketSmem& sm, uint32_t k, uint32_t w, const uint64_t* __restrict__ off,
                                              const uint32_t* __restrict__ ids, uint32_t max_terms,
                                              const uint8_t* __restrict__ dig, const G1Aff* __restrict__ pts,
                                              G1Xyzz* __restrict__ Sb) {
  const Fq S = bucket_sum_q(sm, k, w, off, ids, max_terms, dig, pts);
  const int c = threadIdx.x & 3, b = threadIdx.x >> 2;
  quad::st(Sb + ((size_t)k * kQB + b) * kQW + w, c, fe_canon2p(S));
}

// Window sums for a host Horner (round 5, msm_batch_windows_host): one 256-thread block per (MSM,
// window), 16 lanes per bucket.  Lane l of bucket b sums every 16th entry of the bucket (from the
// l-th) with mixed additions: a chain of at most ceil(n_b / 16) -- the top window of a 128-bit GLV
// half holds 2-3 bits, so its entries crowd into 3-4 buckets, and with 4 lanes per bucket its
// chain of ~10 additions set the kernel time (149 us for create_proof's two 64-term MSMs).  The 16
// partial sums of a bucket go to quad form (4 quads) and add in two levels; then
// sum_b (b + 1) S_b = sum_k 2^k U_k with U_k the sum of the S_b whose digit magnitude d = b + 1 has
// bit k set -- eight buckets each for k < 4 (a quad adds two, then two levels inside its 16-lane
// row), U_4 = S_15 -- on wave 0.  Every quad addition runs through ONE call site (a loop over the
// steps), so the code a wave fetches stays small.  The host places U_k at exponent 5 w + k of one
// Horner.
constexpr int kUPerWin = kQC;  // U_0 .. U_4
constexpr int kUwThreads = 256, kUL = kUwThreads / kQB;  // 16 lanes per bucket
__global__ void __launch_bounds__(kUwThreads) k_batch_uwin(const uint64_t* __restrict__ off, uint32_t max_terms,
                                                           const uint8_t* __restrict__ dig, const G1Aff* __restrict__ pts,
                                                           G1Xyzz* __restrict__ U) {
  __shared__ BucketSmem sm;
  __shared__ Fq sb[kQB][4];
  const uint32_t k = blockIdx.x, w = blockIdx.y, t = threadIdx.x;
  const uint32_t m = (uint32_t)(off[k + 1] - off[k]);
  const uint8_t* dg = dig + ((size_t)k * kQW + w) * 2 * (size_t)max_terms;
  // LDS counting sort of the window's 2m digits by bucket
  if (t < kQB) sm.cnt[t] = 0;
  __syncthreads();
  for (uint32_t j = t; j < 2 * m; j += kUwThreads) {
    const uint32_t d = dg[j];
    if (d & 0x7f) atomicAdd(&sm.cnt[(d & 0x7f) - 1], 1u);
  }
  __syncthreads();
  if (t == 0) {
    uint32_t a = 0;
    for (int bb = 0; bb < kQB; bb++) {
      sm.start[bb] = a;
      a += sm.cnt[bb];
      sm.cnt[bb] = sm.start[bb];
    }
    sm.start[kQB] = a;
  }
  __syncthreads();
  for (uint32_t j = t; j < 2 * m; j += kUwThreads) {
    const uint32_t d = dg[j];
    if (d & 0x7f) sm.lst[atomicAdd(&sm.cnt[(d & 0x7f) - 1], 1u)] = (uint16_t)(j | ((d >> 7) << 15));
  }
  __syncthreads();
  const int b = t / kUL, l = t % kUL, c = t & 3;
  const G1Aff* pk = pts + 2 * (size_t)k * max_terms;
  G1Xyzz acc = G1Xyzz::identity();
  for (uint32_t e = sm.start[b] + l; e < sm.start[b + 1]; e += kUL) {
    const uint32_t v = sm.lst[e];
    const uint32_t* pp = reinterpret_cast<const uint32_t*>(pk + (v & 0x7fff));
    const Fq x = ld_fq(pp);
    Fq y = ld_fq(pp + 8);
    if (x.is_zero() && y.is_zero()) continue;  // identity base
    if (v >> 15) y = -y;
    acc = xyzz_madd_2p(acc, x, y);
  }
  Fq q[4] = {acc.X, acc.Y, acc.ZZ, acc.ZZZ};
  quad::transpose(q, c);  // lane c: coordinate c of the quad's four partial sums
  // steps 0-2: a quad's four sums; 3, 4: + quad qb + 2 (qb < 2), + quad qb + 1 (qb = 0) inside the
  // bucket's 16 lanes; then S_b through LDS; 5: U_kk's members j, j + 4; 6, 7: two levels inside
  // the 16-lane row (wave 0 only from step 5 on)
  const int qb = l >> 2;                           // quad of the bucket
  const int kk = (t >> 2) >> 2, j = (t >> 2) & 3;  // wave 0, quad (kk, j): members j and j + 4 of U_kk
  auto member = [&](int i) {                       // the i-th magnitude with bit kk set, as its bucket index
    return ((((i >> kk) << (kk + 1)) | (1 << kk) | (i & ((1 << kk) - 1))) - 1);
  };
  Fq x = q[0], S15 = q[0];
#pragma unroll 1
  for (int step = 0; step < 8; step++) {
    Fq y;
    if (step < 3) {
      y = quad::pick(step == 0, q[1], quad::pick(step == 1, q[2], q[3]));
    } else if (step < 5) {
      y = quad::down(x, step == 3 ? 8 : 4);  // every shuffle runs on every lane
    } else if (step == 5) {
      if (qb == 0) sb[b][c] = x;  // S_b
      __syncthreads();
      if (t >= 64) break;  // wave-uniform: the U stage runs on wave 0
      S15 = sb[kQB - 1][c];
      x = sb[member(j)][c];
      y = sb[member(j + 4)][c];
    } else {
      y = quad::down(x, step == 6 ? 8 : 4);
    }
    const Fq r = quad::add_2p(x, y, c);
    const bool take = step < 3 || (step == 3 && qb < 2) || (step == 4 && qb == 0) || step == 5 ||
                      (step == 6 && j < 2) || (step == 7 && j == 0);  // quad-uniform
    x = quad::pick(take, r, x);
  }
  if (t >= 64) return;
  G1Xyzz* dst = U + ((size_t)k * kQW + w) * kUPerWin;
  if (j == 0) quad::st(dst + kk, c, fe_canon2p(x));
  if (t < 4) quad::st(dst + 4, c, fe_canon2p(S15));  // U_4 = S_15 (magnitude 16)
}

// Bounded wait for a window's bucket sums (fused kernel): a wave that never sees the flag (a bug,
// not a schedule: see k_batch_fused) raises error bit 8 and goes on, so the grid always drains
__device__ __forceinline__ void wait_ready(const uint32_t* f, uint32_t* err, uint32_t spin_max) {
  uint32_t spins = 0;
  while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
    __builtin_amdgcn_s_sleep(8);
    if (++spins > spin_max) {
      if (threadIdx.x == 0) atomicOr(err, 8u);
      break;
    }
  }
}

// horner_msm: one wave per MSM, quad b runs H_b = sum_w 2^(5w) S_wb (Horner, the next window's sum
// loaded before the doublings), then sum_b (b + 1) H_b = sum_b R_b over the suffix sums R_b (scan
// + tree as k_batch_windows_q), affine on lane 0.  kWait: window w's sums are produced by the same
// launch (k_batch_fused), wait for its flag first.
template <bool kWait>
__device__ __forceinline__ void horner_msm(uint32_t k, const G1Xyzz* __restrict__ Sb, const uint32_t* __restrict__ ids,
                                           int mont, G1Aff* __restrict__ out, const uint32_t* ready,
                                           uint32_t* err, uint32_t spin_max) {
  const int c = threadIdx.x & 3, b = threadIdx.x >> 2;
  const uint32_t id = ids ? ids[k] : k;
  const G1Xyzz* S = Sb + ((size_t)k * kQB + b) * kQW;
  if (kWait) wait_ready(ready + (size_t)k * kQW + kQW - 1, err, spin_max);
  Fq acc = quad::ld(S + kQW - 1, c);
#pragma unroll 1
  for (int w = kQW - 2; w >= 0; w--) {
    if (kWait) wait_ready(ready + (size_t)k * kQW + w, err, spin_max);
    const Fq nxt = quad::ld(S + w, c);
#pragma unroll 1
    for (int i = 0; i < kQC; i++) acc = quad::dbl_2p(acc, c);
    acc = quad::add_2p(acc, nxt, c);
  }
#pragma unroll
  for (int dq = 1; dq < kQB; dq <<= 1) {
    const Fq o = quad::down(acc, 4 * dq);
    if (b + dq < kQB) acc = quad::add_2p(acc, o, c);
  }
#pragma unroll
  for (int dq = kQB / 2; dq >= 1; dq >>= 1) {
    const Fq o = quad::down(acc, 4 * dq);
    if (b < dq) acc = quad::add_2p(acc, o, c);
  }
  const G1Xyzz r = xyzz_canon2p(quad::gather(acc));
  if (threadIdx.x != 0) return;
  G1Aff a = xyzz_to_affine(r);
  if (!mont && !r.is_identity()) {
    a.x = fe_from_mont(a.x);
    a.y = fe_from_mont(a.y);
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(out + id);
  st_fq(o, a.x);
  st_fq(o + 8, a.y);
}

__global__ void __launch_bounds__(64) k_batch_buckets_q(const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ ids, uint32_t max_terms,
                                                        const uint8_t* __restrict__ dig,
                                                        const G1Aff* __restrict__ pts, G1Xyzz* __restrict__ Sb) {
  __shared__ BucketSmem sm;
  bucket_window(sm, blockIdx.x, blockIdx.y, off, ids, max_terms, dig, pts, Sb);
}

__global__ void __launch_bounds__(64) k_batch_horner_b(const G1Xyzz* __restrict__ Sb,
                                                       const uint32_t* __restrict__ ids, int mont,
                                                       G1Aff* __restrict__ out) {
  horner_msm<false>(blockIdx.x, Sb, ids, mont, out, nullptr, nullptr, 0);
}

// Both in ONE launch, so the Horner (the batch's latency floor: ~475 dependent product levels) runs
// while the bucket sums are still being produced: blocks [0, count) are the Horner waves (issued
// first, raised issue priority), then bw bucket waves per MSM, wave j summing windows 25 - j,
// 25 - j - bw, ... in the order the Horner consumes them.  (One block per (MSM, window) makes every
// window finish at about the same time, ~0.27 ms in, and the Horner then starts from scratch.)  A bucket block publishes its window with a release flag; a Horner
// wave waits for each window with an acquire load.  The host only takes this path while the
// Horner waves are a small fraction of the resident-wave capacity (count <= kFuseMax), so bucket
// blocks always find slots and every wait ends.
constexpr uint32_t kFuseMax = 512;

__global__ void __launch_bounds__(64) k_batch_fused(const uint64_t* __restrict__ off, const uint32_t* __restrict__ ids,
                                                    uint32_t count, uint32_t max_terms,
                                                    const uint8_t* __restrict__ dig, const G1Aff* __restrict__ pts,
                                                    G1Xyzz* __restrict__ Sb, uint32_t* ready, uint32_t* err,
                                                    int mont, G1Aff* __restrict__ out, uint32_t bw,
                                                    uint32_t spin_max) {
  __shared__ BucketSmem sm;
  if (blockIdx.x < count) {
    __builtin_amdgcn_s_setprio(3);
    horner_msm<true>(blockIdx.x, Sb, ids, mont, out, ready, err, spin_max);
    return;
  }
  const uint32_t i = blockIdx.x - count;
  const uint32_t k = i % count;
  for (int w = kQW - 1 - (int)(i / count); w >= 0; w -= (int)bw) {
    __syncthreads();
    bucket_window(sm, k, (uint32_t)w, off, ids, max_terms, dig, pts, Sb);
    __threadfence();
    if (threadIdx.x == 0)
      __hip_atomic_store(ready + (size_t)k * kQW + w, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---- Step 3: Horner over the window sums with the independent products of each XYZZ doubling /
// addition issued by up to 4 lanes of one wave at once (LDS slots; 3 product levels per
// doubling instead of 9 products, 4 per addition instead of 14).  One wave per MSM.
enum Slot {
  sX, sY, sZZ, sZZZ,      // accumulator
  tX, tY, tZZ, tZZZ,      // addend
  sU, sV, sX2, sM, sW, sS, sMsq, sX3, sTm, sZZn, sZZZn, sWY, sMS,
  sU1, sU2, sS1, sS2, sP, sR, sPP, sRR, sZ12, sZ123, sPPP, sQ,
  kSlots
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// lanes 0..n-1: R[d_l] = R[a_l] * R[b_l]
__device__ __forceinline__ void par_mul(Fq* R, int lane, int n, int a0, int b0, int d0, int a1 = 0, int b1 = 0,
                                        int d1 = 0, int a2 = 0, int b2 = 0, int d2 = 0, int a3 = 0, int b3 = 0,
                                        int d3 = 0) {
  if (lane < n) {
    const int a = lane == 0 ? a0 : lane == 1 ? a1 : lane == 2 ? a2 : a3;
    const int b = lane == 0 ? b0 : lane == 1 ? b1 : lane == 2 ? b2 : b3;
    const int d = lane == 0 ? d0 : lane == 1 ? d1 : lane == 2 ? d2 : d3;
    const Fq r = R[a] * R[b];
    R[d] = r;
  }
  wave_sync();
}

// dbl-2008-s-1 (same formulas as xyzz_dbl); identity (ZZ = 0) stays identity
__device__ void par_dbl(Fq* R, int lane) {
  if (lane == 0) R[sU] = fe_dbl(R[sY]);
  wave_sync();
  par_mul(R, lane, 2, sU, sU, sV, sX, sX, sX2);
  if (lane == 0) R[sM] = fe_dbl(R[sX2]) + R[sX2];
  wave_sync();
  par_mul(R, lane, 4, sU, sV, sW, sX, sV, sS, sV, sZZ, sZZn, sM, sM, sMsq);
  if (lane == 0) {
    const Fq x3 = R[sMsq] - fe_dbl(R[sS]);
    R[sX3] = x3;
    R[sTm] = R[sS] - x3;
  }
  wave_sync();
  par_mul(R, lane, 3, sW, sZZZ, sZZZn, sW, sY, sWY, sM, sTm, sMS);
  if (lane == 0) {
    R[sY] = R[sMS] - R[sWY];
    R[sX] = R[sX3];
    R[sZZ] = R[sZZn];
    R[sZZZ] = R[sZZZn];
  }
  wave_sync();
}

// add-2008-s: acc += addend (slots t*), complete (identities, P == Q, P == -Q)
__device__ void par_add(Fq* R, int lane) {
  if (R[tZZ].is_zero()) return;  // LDS broadcast reads: uniform branches
  if (R[sZZ].is_zero()) {
    if (lane == 0) {
      R[sX] = R[tX];
      R[sY] = R[tY];
      R[sZZ] = R[tZZ];
      R[sZZZ] = R[tZZZ];
    }
    wave_sync();
    return;
  }
  par_mul(R, lane, 4, sX, tZZ, sU1, tX, sZZ, sU2, sY, tZZZ, sS1, tY, sZZZ, sS2);
  if (lane == 0) {
    R[sP] = R[sU2] - R[sU1];
    R[sR] = R[sS2] - R[sS1];
  }
  wave_sync();
  if (R[sP].is_zero()) {
    if (R[sR].is_zero()) {
      par_dbl(R, lane);
    } else {
      if (lane == 0) R[sZZ] = R[sZZZ] = Fq::zero();
      wave_sync();
    }
    return;
  }
  par_mul(R, lane, 4, sP, sP, sPP, sR, sR, sRR, sZZ, tZZ, sZ12, sZZZ, tZZZ, sZ123);
  par_mul(R, lane, 3, sP, sPP, sPPP, sU1, sPP, sQ, sZ12, sPP, sZZn);
  if (lane == 0) {
    const Fq x3 = R[sRR] - R[sPPP] - fe_dbl(R[sQ]);
    R[sX3] = x3;
    R[sTm] = R[sQ] - x3;
  }
  wave_sync();
  par_mul(R, lane, 3, sR, sTm, sMS, sS1, sPPP, sWY, sZ123, sPPP, sZZZn);
  if (lane == 0) {
    R[sY] = R[sMS] - R[sWY];
    R[sX] = R[sX3];
    R[sZZ] = R[sZZn];
    R[sZZZ] = R[sZZZn];
  }
  wave_sync();
}

template <int C>
__global__ void __launch_bounds__(64) k_msm_batch_horner(const G1Xyzz* __restrict__ Tg, const uint32_t* __restrict__ ids,
                                                         int mont, G1Aff* __restrict__ out) {
  constexpr int W = BatchCfg<C>::W;
  __shared__ Fq R[kSlots];
  const int lane = threadIdx.x;
  const uint32_t id = ids ? ids[blockIdx.x] : blockIdx.x;
  const G1Xyzz* T = Tg + (size_t)blockIdx.x * W;
  if (lane == 0) {
    const G1Xyzz t = T[W - 1];
    R[sX] = t.X, R[sY] = t.Y, R[sZZ] = t.ZZ, R[sZZZ] = t.ZZZ;
  }
  wave_sync();
  for (int w = W - 2; w >= 0; w--) {
    for (int i = 0; i < C; i++) par_dbl(R, lane);
    if (lane == 0) {
      const G1Xyzz t = T[w];
      R[tX] = t.X, R[tY] = t.Y, R[tZZ] = t.ZZ, R[tZZZ] = t.ZZZ;
    }
    wave_sync();
    par_add(R, lane);
  }
  if (lane == 0) {
    const G1Xyzz acc = {R[sX], R[sY], R[sZZ], R[sZZZ]};
    G1Aff r = xyzz_to_affine(acc);
    if (!mont && !acc.is_identity()) {
      r.x = fe_from_mont(r.x);
      r.y = fe_from_mont(r.y);
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out + id);
    st_fq(o, r.x);
    st_fq(o + 8, r.y);
  }
}

// ---- Step 3, quad form (default): one QUAD of lanes per MSM (quad.hpp: lane c holds coordinate c),
// 16 MSMs per wave; a doubling is 3 product levels and an addition 4, operands moved by DPP inside
// the quad -- no LDS slots and no wave-wide syncs, and the batch runs 16 chains per wave instead
// of one.  The lanes of a quad share every branch (quad-uniform), so DPP always reads live lanes.
template <int C>
__global__ void __launch_bounds__(64) k_msm_batch_horner_q(const G1Xyzz* __restrict__ Tg,
                                                           const uint32_t* __restrict__ ids, uint32_t count,
                                                           int mont, G1Aff* __restrict__ out) {
  constexpr int W = BatchCfg<C>::W;
  const int c = threadIdx.x & 3;
  const uint32_t qi = blockIdx.x * 16 + (threadIdx.x >> 2);
  if (qi >= count) return;  // uniform within the quad
  const uint32_t id = ids ? ids[qi] : qi;
  const G1Xyzz* T = Tg + (size_t)qi * W;
  Fq acc = quad::ld(T + W - 1, c);
#pragma unroll 1
  for (int w = W - 2; w >= 0; w--) {
    const Fq nxt = quad::ld(T + w, c);  // in flight during the doublings
#pragma unroll 1
    for (int i = 0; i < C; i++) acc = quad::dbl_2p(acc, c);
    acc = quad::add_2p(acc, nxt, c);
  }
  const G1Xyzz r = xyzz_canon2p(quad::gather(acc));
  if (c != 0) return;
  G1Aff a = xyzz_to_affine(r);
  if (!mont && !r.is_identity()) {
    a.x = fe_from_mont(a.x);
    a.y = fe_from_mont(a.y);
  }
  uint32_t* o = reinterpret_cast<uint32_t*>(out + id);
  st_fq(o, a.x);
  st_fq(o + 8, a.y);
}

// ---- Precomputed fixed bases (base tables) -------------------------------------
// A table row P is stored as its window multiples Q_w = 2^(8 w) P, w < kFixW (affine, Montgomery),
// so sum_i k_i P_i = sum_i sum_w d_iw Q_iw: every signed 8-bit digit of every term lands in ONE set
// of 128 buckets and the per-MSM Horner chain over windows disappears.  One 256-thread block per
// MSM: digits -> LDS counting sort by bucket (chunks of kFixChunk terms), two threads per bucket
// sum their half of its entries with mixed adds, then sum_b (b + 1) S_b = sum_k T_k over the
// suffix sums T_k = sum_{b >= k} S_b: a 7-level LDS scan and a 7-level tree (depth 14 instead of the
// ~128 dependent doublings of the window Horner), and one inversion for the affine output.
constexpr int kFixC = 8;
constexpr int kFixB = 1 << (kFixC - 1);                  // 128 buckets (signed digits)
constexpr int kFixW = (255 + kFixC - 1) / kFixC;         // 32 windows cover scalars < r < 2^254
constexpr int kFixChunk = 256;                           // terms per LDS pass

// one thread per row: Q_w = 2^(8 w) P (identity rows stay (0, 0))
__global__ void __launch_bounds__(kThreads) k_table_precompute(const G1Aff* __restrict__ rows, uint32_t n,
                                                               G1Aff* __restrict__ pre) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* rp = reinterpret_cast<const uint32_t*>(rows + i);
  const Fq x = ld_fq(rp), y = ld_fq(rp + 8);
  uint32_t* o = reinterpret_cast<uint32_t*>(pre + (size_t)i * kFixW);
  if (x.is_zero() && y.is_zero()) {
    for (int w = 0; w < kFixW; w++) {
      st_fq(o + 16 * w, Fq::zero());
      st_fq(o + 16 * w + 8, Fq::zero());
    }
    return;
  }
  G1Xyzz acc = {x, y, Fq::one(), Fq::one()};
  for (int w = 0; w < kFixW; w++) {
    if (w) {
      for (int d = 0; d < kFixC; d++) acc = xyzz_dbl(acc);
    }
    const G1Aff a = xyzz_to_affine(acc);  // never the identity: P has prime order r > 2^(8 w)
    st_fq(o + 16 * w, a.x);
    st_fq(o + 16 * w + 8, a.y);
  }
}

__global__ void __launch_bounds__(kThreads) k_msm_batch_fixed(const G1Aff* __restrict__ pre, uint32_t rows,
                                                              const uint32_t* __restrict__ bidx,
                                                              const Fr* __restrict__ scalars,
                                                              const uint64_t* __restrict__ off, int mont,
                                                              G1Aff* __restrict__ out, uint32_t* __restrict__ err) {
  __shared__ uint32_t cnt[kFixB];                 // histogram, then scatter cursors
  __shared__ uint32_t bst[kFixB + 1];             // bucket starts in lst
  __shared__ uint32_t lst[kFixChunk * kFixW];     // (row * kFixW + w) << 1 | sign, sorted by bucket
  __shared__ uint8_t dig[kFixChunk * kFixW];      // magnitude of digit (term, w); sign in sgn
  __shared__ uint32_t sgn[kFixChunk];             // sign bits of the term's kFixW digits
  __shared__ G1Xyzz T[kFixB];
  const int tid = threadIdx.x;
  const uint32_t id = blockIdx.x;
  const uint64_t b0 = off[id], e0 = off[id + 1];
  const int bucket = tid % kFixB, part = tid / kFixB;  // 2 threads per bucket
  G1Xyzz acc = G1Xyzz::identity();
  for (uint64_t c0 = b0; c0 < e0; c0 += kFixChunk) {
    const int m = (int)(e0 - c0 < (uint64_t)kFixChunk ? e0 - c0 : (uint64_t)kFixChunk);
    if (tid < kFixB) cnt[tid] = 0;
    __syncthreads();
    uint32_t row = 0;
    if (tid < m) {
      Fr s;
      {
        const Fq t = ld_fq(reinterpret_cast<const uint32_t*>(scalars + c0 + tid));
#pragma unroll
        for (int i = 0; i < 8; i++) s.v[i] = t.v[i];
      }
      if (!s.is_reduced()) atomicOr(err, 2u);
      if (mont) s = fe_from_mont(s);
      row = bidx[c0 + tid];
      if (row >= rows) {
        atomicOr(err, 4u);
        s = Fr::zero();
      }
      uint32_t carry = 0, sg = 0;
      for (int w = 0; w < kFixW; w++) {  // signed 8-bit digits in (-128, 128]
        const uint32_t bits = ((s.v[w >> 2] >> ((w & 3) * 8)) & 0xffu) + carry;
        uint32_t mag;
        if (bits > (uint32_t)kFixB) {
          mag = 256u - bits;  // bits == 256: digit 0, carry 1
          if (mag) sg |= 1u << w;
          carry = 1;
        } else {
          mag = bits;
          carry = 0;
        }
        dig[tid * kFixW + w] = (uint8_t)mag;
        if (mag) atomicAdd(&cnt[mag - 1], 1u);
      }
      sgn[tid] = sg;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t a = 0;
      for (int b = 0; b < kFixB; b++) {
        bst[b] = a;
        a += cnt[b];
        cnt[b] = bst[b];
      }
      bst[kFixB] = a;
    }
    __syncthreads();
    if (tid < m) {
      const uint32_t sg = sgn[tid];
      for (int w = 0; w < kFixW; w++) {
        const uint32_t mag = dig[tid * kFixW + w];
        if (mag) lst[atomicAdd(&cnt[mag - 1], 1u)] = ((row * kFixW + w) << 1) | ((sg >> w) & 1u);
      }
    }
    __syncthreads();
    for (uint32_t q = bst[bucket] + part; q < bst[bucket + 1]; q += 2) {
      const uint32_t e = lst[q];
      const uint32_t* qp = reinterpret_cast<const uint32_t*>(pre + (e >> 1));
      G1Aff a;
      a.x = ld_fq(qp);
      a.y = ld_fq(qp + 8);
      if (a.x.is_zero() && a.y.is_zero()) continue;  // identity row
      if (e & 1) a.y = -a.y;
      acc = xyzz_madd_2p(acc, a.x, a.y);  // the bucket sums stay in the 2p domain (curve.hpp)
    }
    __syncthreads();
  }
  // S_b = the two halves of bucket b
  if (part == 1) T[bucket] = acc;
  __syncthreads();
  if (part == 0) T[bucket] = xyzz_add_2p(acc, T[bucket]);
  __syncthreads();
  // suffix sums T_k = sum_{b >= k} S_b (Hillis-Steele, 7 levels)
  for (int d = 1; d < kFixB; d <<= 1) {
    G1Xyzz v = G1Xyzz::identity();
    const bool live = tid < kFixB && tid + d < kFixB;
    if (live) v = T[tid + d];
    __syncthreads();
    if (live) T[tid] = xyzz_add_2p(T[tid], v);
    __syncthreads();
  }
  // sum_b (b + 1) S_b = sum_k T_k (tree, 7 levels)
  for (int h = kFixB / 2; h >= 1; h >>= 1) {
    if (tid < h) T[tid] = xyzz_add_2p(T[tid], T[tid + h]);
    __syncthreads();
  }
  if (tid == 0) {
    const G1Xyzz r = xyzz_canon2p(T[0]);
    G1Aff a = xyzz_to_affine(r);
    if (!mont && !r.is_identity()) {
      a.x = fe_from_mont(a.x);
      a.y = fe_from_mont(a.y);
    }
    uint32_t* o = reinterpret_cast<uint32_t*>(out + id);
    st_fq(o, a.x);
    st_fq(o + 8, a.y);
  }
}

}  // namespace

static std::atomic<uint64_t> g_fused_redone{0};  // fused launches redone by the two-kernel path

int msm_batch_window_bits(size_t max_terms) {
  if (const char* e = getenv("SVGPU_BATCH_WINDOW_BITS")) {
    const int c = atoi(e);
    if (c == 5 || c == 8) return c;
  }
  return max_terms <= 256 ? 5 : 8;
}

// Small plain batches (round 5): the window sums on the device and one host Horner per MSM on the
// host pool (msm_batch_windows_host) instead of the fused kernel, whose one-wave Horner chain takes
// ~0.65 ms whatever the batch size (one 64-term MSM as long as 128 of them,
// profiles/r05_batch_floor_probe.log).  The host costs ~35 us per MSM, spread over the pool:
// 0.17-0.20 ms for 1-16 MSMs of 64 terms, 0.47 at 64, even at ~100, slower at 128
// (profiles/r05_batch_host_route_ab.log).  SVGPU_BATCH_HOST_MAX sets the largest such batch (0: never).
constexpr size_t kBatchHostMax = 64;
static int msm_batch_small_host(const void* d_bases, const void* d_scalars, const uint64_t* d_offsets, size_t count,
                                size_t max_terms, int form, int device, hipStream_t stream, void* d_out) {
  std::vector<host::Xyzz> acc(count);
  SV_TRY(msm_batch_windows_host(d_bases, d_scalars, d_offsets, count, max_terms, form, form, device, stream,
                                acc.data()));
  // affine in `form` with ONE inversion (Montgomery's trick over the ZZZ of the non-identity sums):
  // x = X / ZZ = X (ZZ ZZZ^-1)^2, y = Y / ZZZ; the identity is (0, 0)
  std::vector<host::F> pre(count);
  host::F run = host::f_one();
  for (size_t k = 0; k < count; k++) {
    pre[k] = run;  // product of the earlier non-identity ZZZ
    if (!host::x_is_identity(acc[k])) run = host::f_mul(run, acc[k].ZZZ);
  }
  host::F inv = host::f_inv(run);
  std::vector<uint64_t> h(8 * count, 0);
  for (size_t k = count; k-- > 0;) {
    if (host::x_is_identity(acc[k])) continue;
    const host::F izzz = host::f_mul(inv, pre[k]);
    inv = host::f_mul(inv, acc[k].ZZZ);
    const host::F iz = host::f_mul(izzz, acc[k].ZZ);
    host::F x = host::f_mul(acc[k].X, host::f_sqr(iz)), y = host::f_mul(acc[k].Y, izzz);
    if (form != SV_MONTGOMERY) x = host::f_from_mont(x), y = host::f_from_mont(y);
    memcpy(&h[8 * k], x.l, 32);
    memcpy(&h[8 * k + 4], y.l, 32);
  }
  // on the caller's stream (no null-stream implicit sync); this route is synchronous for the host
  // anyway (msm_batch_windows_host waited for the window sums), so wait for the copy of `h`
  SV_HIP(hipSetDevice(device));
  SV_HIP(hipMemcpyAsync(d_out, h.data(), h.size() * 8, hipMemcpyHostToDevice, stream));
  SV_HIP(hipStreamSynchronize(stream));
  return SV_OK;
}

int msm_batch_device(const void* d_bases, const void* d_scalars, const uint64_t* d_offsets, const uint32_t* d_ids,
                     size_t count, size_t max_terms, int form, int device, hipStream_t stream, void* d_out,
                     const uint32_t* d_bidx, uint64_t table_len, int base_form) {
  if (count == 0) return SV_OK;
  if (count > 0x7fffffffull) {
    set_error("msm_batch: count = %zu too large", count);
    return SV_ERR_LEN;
  }
  {
    const char* hm = getenv("SVGPU_BATCH_HOST_MAX");  // read per call
    const size_t host_max = hm ? (size_t)strtoull(hm, nullptr, 10) : kBatchHostMax;
    if (!d_ids && !d_bidx && count <= host_max && max_terms >= 1 && max_terms <= (size_t)kQMaxTerms &&
        msm_batch_window_bits(max_terms) == kQC)
      return msm_batch_small_host(d_bases, d_scalars, d_offsets, count, max_terms, form, device, stream, d_out);
  }
  WsLease lease(device, stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  hipStream_t st = ws->stream;
  const int c = msm_batch_window_bits(max_terms);
  const int W = c == 5 ? BatchCfg<5>::W : BatchCfg<8>::W;
  const int WG = c == 5 ? BatchCfg<5>::WG : BatchCfg<8>::WG;
  // SVGPU_BATCH_QUAD=0: the round-2 kernels (per-lane window sums, one-wave Horner)
  const bool quad_path = !getenv("SVGPU_BATCH_QUAD") || atoi(getenv("SVGPU_BATCH_QUAD")) != 0;
  const bool quad_windows = quad_path && c == kQC && max_terms <= (size_t)kQMaxTerms;
  // bucket-wise Horner (k_batch_buckets_q + k_batch_horner_b; SVGPU_BATCH_BUCKETS=0 keeps the
  // per-window weighting of k_batch_windows_q): 16 bucket sums per window instead of one window sum,
  // 53 KB per MSM, so very large batches keep the per-window path
  const bool bucket_horner = quad_windows && count <= 4096 &&
                             (!getenv("SVGPU_BATCH_BUCKETS") || atoi(getenv("SVGPU_BATCH_BUCKETS")) != 0);
  const size_t dig_bytes = quad_windows ? count * kQW * 2 * max_terms : 0;
  const size_t pts_bytes = quad_windows ? count * 2 * max_terms * sizeof(G1Aff) : 0;
  const size_t nT = bucket_horner ? count * kQB * kQW : count * W;
  // one launch for buckets + Horner while the Horner waves stay few (k_batch_fused; SVGPU_BATCH_FUSE=0
  // runs the two kernels back to back)
  // HIP promises no co-residency between workgroups of a launch, and the Horner waves of a fused
  // launch hold their slots while they wait: one fused launch (count <= kFuseMax waves) leaves most
  // of the chip's wave slots to its bucket blocks, but several at once on one GPU (concurrent
  // callers, SVGPU_DEVICE_MAP repeats) could fill it with waiting waves.  So at most ONE fused launch
  // is in flight per physical device; the others take the two-kernel path.  A launch whose wait
  // times out anyway (error bit 8) is redone below by the two-kernel path, never reported.
  bool fused = bucket_horner && count <= kFuseMax &&
               (!getenv("SVGPU_BATCH_FUSE") || atoi(getenv("SVGPU_BATCH_FUSE")) != 0);
  struct FuseSlot {
    std::atomic<int>* slot = nullptr;
    ~FuseSlot() {
      if (slot) slot->fetch_sub(1, std::memory_order_acq_rel);
    }
  } fuse_slot;
  if (fused) {
    static std::atomic<int> inflight[64];
    std::atomic<int>& f = inflight[device & 63];
    if (f.fetch_add(1, std::memory_order_acq_rel) == 0) {
      fuse_slot.slot = &f;
    } else {
      f.fetch_sub(1, std::memory_order_acq_rel);
      fused = false;
    }
  }
  const size_t nflag = fused ? count * kQW : 0;
  SV_TRY(ws->reserve(Workspace::aligned(4 * (1 + nflag)) + Workspace::aligned(nT * sizeof(G1Xyzz)) +
                     Workspace::aligned(dig_bytes ? dig_bytes : 1) + Workspace::aligned(pts_bytes ? pts_bytes : 1)));
  SV_TRY(ws->reserve_pinned(256));
  uint32_t* err = ws->carve<uint32_t>(1 + nflag);  // the error word, then the window flags
  G1Xyzz* Tg = ws->carve<G1Xyzz>(nT);
  uint8_t* dig = ws->carve<uint8_t>(dig_bytes ? dig_bytes : 1);
  G1Aff* pts = ws->carve<G1Aff>(pts_bytes ? pts_bytes / sizeof(G1Aff) : 1);
  SV_HIP(hipMemsetAsync(err, 0, 4 * (1 + nflag), st));
  const int mont = form == SV_MONTGOMERY;
  const int mont_b = (d_bidx ? base_form : form) == SV_MONTGOMERY;
  const G1Aff* b = static_cast<const G1Aff*>(d_bases);
  const Fr* s = static_cast<const Fr*>(d_scalars);
  G1Aff* o = static_cast<G1Aff*>(d_out);
  const dim3 grid((uint32_t)count, WG);
  const bool quad_horner = quad_path;
  if (quad_windows) {
    hipLaunchKernelGGL(k_batch_prep, dim3((uint32_t)count, (uint32_t)((max_terms + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, st, b, s, d_offsets, d_ids, mont, (uint32_t)max_terms, dig, pts, err, d_bidx,
                       table_len, mont_b);
    if (fused) {
      // SVGPU_BATCH_WAIT_SPINS: the wait bound (default 2^22 sleeps, ~1 s); tests set it to 0 to
      // force the timeout and the two-kernel redo
      const char* spins_env = getenv("SVGPU_BATCH_WAIT_SPINS");
      const uint32_t spin_max = spins_env ? (uint32_t)strtoul(spins_env, nullptr, 10) : (1u << 22);
      const uint32_t bw = std::min<uint32_t>(kQW, std::max(1, getenv("SVGPU_BATCH_BW") ? atoi(getenv("SVGPU_BATCH_BW")) : 4));
      hipLaunchKernelGGL(k_batch_fused, dim3((uint32_t)(count * (1 + bw))), dim3(64), 0, st, d_offsets, d_ids,
                         (uint32_t)count, (uint32_t)max_terms, dig, pts, Tg, err + 1, err, mont, o, bw, spin_max);
    } else if (bucket_horner) {
      hipLaunchKernelGGL(k_batch_buckets_q, dim3((uint32_t)count, (uint32_t)kQW), dim3(64), 0, st, d_offsets, d_ids,
                         (uint32_t)max_terms, dig, pts, Tg);
      hipLaunchKernelGGL(k_batch_horner_b, dim3((uint32_t)count), dim3(64), 0, st, Tg, d_ids, mont, o);
    } else {
      hipLaunchKernelGGL(k_batch_windows_q, dim3((uint32_t)count, (uint32_t)kQW), dim3(64), 0, st, d_offsets, d_ids,
                         (uint32_t)max_terms, dig, pts, Tg);
      hipLaunchKernelGGL(k_msm_batch_horner_q<5>, dim3((uint32_t)((count + 15) / 16)), dim3(64), 0, st, Tg, d_ids,
                         (uint32_t)count, mont, o);
    }
  } else if (c == 5) {
    hipLaunchKernelGGL(k_msm_batch_windows<5>, grid, dim3(kThreads), 0, st, b, s, d_offsets, d_ids, mont, Tg, err,
                       d_bidx, table_len, mont_b);
    if (quad_horner)
      hipLaunchKernelGGL(k_msm_batch_horner_q<5>, dim3((uint32_t)((count + 15) / 16)), dim3(64), 0, st, Tg, d_ids,
                         (uint32_t)count, mont, o);
    else
      hipLaunchKernelGGL(k_msm_batch_horner<5>, dim3((uint32_t)count), dim3(64), 0, st, Tg, d_ids, mont, o);
  } else {
    hipLaunchKernelGGL(k_msm_batch_windows<8>, grid, dim3(kThreads), 0, st, b, s, d_offsets, d_ids, mont, Tg, err,
                       d_bidx, table_len, mont_b);
    if (quad_horner)
      hipLaunchKernelGGL(k_msm_batch_horner_q<8>, dim3((uint32_t)((count + 15) / 16)), dim3(64), 0, st, Tg, d_ids,
                         (uint32_t)count, mont, o);
    else
      hipLaunchKernelGGL(k_msm_batch_horner<8>, dim3((uint32_t)count), dim3(64), 0, st, Tg, d_ids, mont, o);
  }
  SV_HIP(hipGetLastError());
  SV_HIP(hipMemcpyAsync(ws->pinned, err, 4, hipMemcpyDeviceToHost, st));
  SV_HIP(hipStreamSynchronize(st));
  uint32_t ev;
  memcpy(&ev, ws->pinned, 4);
  if (ev & 1u) {
    set_error("msm_batch: base coordinate not reduced mod p");
    return SV_ERR_ARG;
  }
  if (ev & 2u) {
    set_error("msm_batch: scalar not reduced (>= r)");
    return SV_ERR_ARG;
  }
  if (ev & 4u) {
    set_error("msm_batch: base index out of the table (>= %llu)", (unsigned long long)table_len);
    return SV_ERR_ARG;
  }
  if (ev & 8u) {
    // a fused launch's Horner wave gave up waiting (the GPU was full of other waves): its outputs
    // are garbage, so redo the bucket sums and the Horner as two ordered launches
    SV_HIP(hipMemsetAsync(err, 0, 4, st));
    hipLaunchKernelGGL(k_batch_buckets_q, dim3((uint32_t)count, (uint32_t)kQW), dim3(64), 0, st, d_offsets, d_ids,
                       (uint32_t)max_terms, dig, pts, Tg);
    hipLaunchKernelGGL(k_batch_horner_b, dim3((uint32_t)count), dim3(64), 0, st, Tg, d_ids, mont, o);
    SV_HIP(hipGetLastError());
    SV_HIP(hipStreamSynchronize(st));
    g_fused_redone.fetch_add(1, std::memory_order_relaxed);
  }
  return SV_OK;
}

uint64_t msm_batch_fused_redone() { return g_fused_redone.load(std::memory_order_relaxed); }

// ---- Small batches with the window Horner on the host (round 5).  A batch of a few MSMs of at most
// kQMaxTerms terms -- KzgAs::create_proof's two r^i MSMs (accumulation.rs:177-192), a native
// verifier's per-proof MSMs -- is bound by its serial tail: the Horner over the 26 windows of a
// 128-bit GLV half (130 doublings) is ~475 dependent product levels on one GPU wave, ~0.25 ms, but
// ~40 us on the host (host_ec.hpp).  The device forms each window's partial sums U_k (k_batch_prep
// + k_batch_uwin), one copy brings them back, the host combines them.
// d_offsets = nullptr: one MSM of max_terms terms.
int msm_batch_windows_host(const void* d_bases, const void* d_scalars, const uint64_t* d_offsets, size_t count,
                           size_t max_terms, int scalar_form, int base_form, int device, hipStream_t stream,
                           host::Xyzz* out) {
  if (count == 0) return SV_OK;
  if (max_terms == 0 || max_terms > (size_t)kQMaxTerms || count > 0xffffu) {
    set_error("msm_batch_windows_host: %zu MSMs of up to %zu terms (at most %d terms)", count, max_terms, kQMaxTerms);
    return SV_ERR_ARG;
  }
  WsLease lease(device, stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  hipStream_t st = ws->stream;
  const size_t nT = count * kQW * kUPerWin;
  const size_t dig_bytes = count * kQW * 2 * max_terms;
  const size_t pts_bytes = count * 2 * max_terms * sizeof(G1Aff);
  const size_t t_off = 256;  // the error word, then the window sums: ONE copy back
  const size_t back = t_off + nT * sizeof(G1Xyzz);  // bytes copied back
  SV_TRY(ws->reserve(t_off + Workspace::aligned(nT * sizeof(G1Xyzz)) + Workspace::aligned(dig_bytes) +
                     Workspace::aligned(pts_bytes) + 256));
  SV_TRY(ws->reserve_pinned(Workspace::aligned(back) + 16));
  unsigned char* blk = ws->carve<unsigned char>(t_off + Workspace::aligned(nT * sizeof(G1Xyzz)));
  uint32_t* err = reinterpret_cast<uint32_t*>(blk);
  G1Xyzz* Tg = reinterpret_cast<G1Xyzz*>(blk + t_off);
  uint8_t* dig = ws->carve<uint8_t>(dig_bytes);
  G1Aff* pts = ws->carve<G1Aff>(pts_bytes / sizeof(G1Aff));
  if (!d_offsets) {  // one MSM of max_terms terms (msm_run_impl's small path): offsets {0, max_terms}
    if (count != 1) return SV_ERR_ARG;
    uint64_t* hoff = reinterpret_cast<uint64_t*>(ws->pinned + Workspace::aligned(back));
    hoff[0] = 0;
    hoff[1] = max_terms;
    uint64_t* doff = ws->carve<uint64_t>(2);
    SV_HIP(hipMemcpyAsync(doff, hoff, 16, hipMemcpyHostToDevice, st));
    d_offsets = doff;
  }
  SV_HIP(hipMemsetAsync(err, 0, 4, st));
  hipLaunchKernelGGL(k_batch_prep, dim3((uint32_t)count, (uint32_t)((max_terms + kThreads - 1) / kThreads)),
                     dim3(kThreads), 0, st, static_cast<const G1Aff*>(d_bases), static_cast<const Fr*>(d_scalars),
                     d_offsets, nullptr, scalar_form == SV_MONTGOMERY ? 1 : 0, (uint32_t)max_terms, dig, pts, err,
                     nullptr, (uint64_t)0, base_form == SV_MONTGOMERY ? 1 : 0);
  hipLaunchKernelGGL(k_batch_uwin, dim3((uint32_t)count, (uint32_t)kQW), dim3(kUwThreads), 0, st, d_offsets,
                     (uint32_t)max_terms, dig, pts, Tg);
  SV_HIP(hipGetLastError());
  SV_HIP(hipMemcpyAsync(ws->pinned, blk, back, hipMemcpyDeviceToHost, st));
  SV_HIP(hipStreamSynchronize(st));
  uint32_t ev;
  memcpy(&ev, ws->pinned, 4);
  if (ev & 1u) {
    set_error("msm_batch: base coordinate not reduced mod p");
    return SV_ERR_ARG;
  }
  if (ev & 2u) {
    set_error("msm_batch: scalar not reduced (>= r)");
    return SV_ERR_ARG;
  }
  // the partial sums are canonical Montgomery XYZZ (host::Xyzz has the same bytes); U_k of window w
  // sits at exponent 5 w + k: one Horner over the 130 exponents per MSM, the MSMs on the host pool
  const host::Xyzz* U = reinterpret_cast<const host::Xyzz*>(ws->pinned + t_off);
  constexpr int kTop = kQW * kUPerWin - 1;
  host_parallel_for(count, 1, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; k++) {
      const host::Xyzz* u = U + k * kQW * kUPerWin;
      host::Xyzz acc = u[kTop];
      for (int e = kTop - 1; e >= 0; e--) acc = host::x_add(host::x_dbl(acc), u[e]);
      out[k] = acc;
    }
  });
  return SV_OK;
}

}  // namespace sv

namespace sv {

size_t table_precomputed_rows_bytes(size_t n) { return n * (size_t)kFixW * sizeof(G1Aff); }

int table_precompute_device(const void* d_rows, size_t n, void* d_pre, int device) {
  if (n == 0) return SV_OK;
  WsLease lease(device, nullptr);
  if (!lease.ok()) return SV_ERR_DEVICE;
  hipStream_t st = lease.get()->stream;
  hipLaunchKernelGGL(k_table_precompute, dim3((uint32_t)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                     static_cast<const G1Aff*>(d_rows), (uint32_t)n, static_cast<G1Aff*>(d_pre));
  SV_HIP(hipGetLastError());
  SV_HIP(hipStreamSynchronize(st));
  return SV_OK;
}

int msm_batch_fixed_device(const void* d_pre, size_t rows, const uint32_t* d_bidx, const void* d_scalars,
                           const uint64_t* d_offsets, size_t count, int form, int device, hipStream_t stream,
                           void* d_out) {
  if (count == 0) return SV_OK;
  if (count > 0x7fffffffull) {
    set_error("msm_batch: count = %zu too large", count);
    return SV_ERR_LEN;
  }
  WsLease lease(device, stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  hipStream_t st = ws->stream;
  SV_TRY(ws->reserve(Workspace::aligned(4)));
  SV_TRY(ws->reserve_pinned(256));
  uint32_t* err = ws->carve<uint32_t>(1);
  SV_HIP(hipMemsetAsync(err, 0, 4, st));
  hipLaunchKernelGGL(k_msm_batch_fixed, dim3((uint32_t)count), dim3(kThreads), 0, st, static_cast<const G1Aff*>(d_pre),
                     (uint32_t)rows, d_bidx, static_cast<const Fr*>(d_scalars), d_offsets,
                     form == SV_MONTGOMERY ? 1 : 0, static_cast<G1Aff*>(d_out), err);
  SV_HIP(hipGetLastError());
  SV_HIP(hipMemcpyAsync(ws->pinned, err, 4, hipMemcpyDeviceToHost, st));
  SV_HIP(hipStreamSynchronize(st));
  uint32_t ev;
  memcpy(&ev, ws->pinned, 4);
  if (ev & 2u) {
    set_error("msm_batch: scalar not reduced (>= r)");
    return SV_ERR_ARG;
  }
  if (ev & 4u) {
    set_error("msm_batch: base index out of the table (>= %zu)", rows);
    return SV_ERR_ARG;
  }
  return SV_OK;
}

}  // namespace sv
