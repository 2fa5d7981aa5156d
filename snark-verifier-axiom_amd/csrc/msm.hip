// Pippenger bucket MSM for BN254 G1 on gfx950.
//
// Replaces util::msm::multi_scalar_multiplication (snark-verifier/src/util/msm.rs:238-316) and
// the naive NativeLoader::multi_scalar_multiplication (snark-verifier/src/loader/native.rs:61-71):
// same group element out, computed as a signed-digit bucket method.
//
// Pipeline (all on one stream, inputs already in HBM):
//   k_to_mont_bases   (canonical input only) bases -> Montgomery workspace copy
//   k_bin_hist        per block of sort_chunk points (1024 at 2^20; XCD-aware block map, sort_block): signed c-bit digits of every
//                     window (digits never stored; the GLV halves are, 32 B per point, for the scatter)
//                     + the point table, LDS
//                     histogram of (window, coarse bin = top bits of the bucket)
//   k_bin_scan_chunks / k_bin_scan   offsets of every (window, bin, block) run
//   k_bin_scatter     digits again (from the stored halves); entries appended to their block's (window, bin) run -> tmp
//   k_fine_sort<2>    one block per (window, bin), both region kinds in one launch: counting sort
//                     by the fine bucket index inside the bin's L2-resident region -> ent[], bucket
//                     offsets gst[], owner bucket of every accumulate chunk tstart[]
//   k_accumulate      each thread sums K consecutive sorted entries (mixed XYZZ adds over 29-bit
//                     limbs by default, points from a table in that form -- see AccChain; perfect
//                     load balance whatever the digit distribution), complete buckets written
//                     directly, bucket pieces that cross a thread boundary to pfirst/plast
//                     (two-piece buckets inside a block are joined at the end through LDS)
//   k_fixup           the other crossing buckets, queued by k_accumulate (heavy ones: block-level
//                     tree for buckets spanning more than 9 threads)
//   k_wsum_tree       bucket reduction: F_w = sum_b (b+1) S_b = sum_j acc_j + L sum_j j T_j with
//                     running sums over segments of L buckets (acc_j, T_j), then sum_j j T_j =
//                     sum_k 2^k U_k, U_k = sum_{j : bit k of j} T_j, as a subset-sum tree over each
//                     block's 256 segments in LDS (round 3; k_wsum + k_group_sum(_q) below for
//                     windows of fewer than 256 segments)
//   k_group_fin       the blocks' partial sums -> A and U_k per window
//   host              ONE Horner over every (window, bit) exponent -> affine, see host_ec.hpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <functional>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "curve.hpp"
#include "curve29.hpp"
#include "glv.hpp"
#include "host_ec.hpp"
#include "msm.hpp"
#include "msm_batch.hpp"
#include "quad.hpp"
#include "runtime.hpp"

namespace sv {

static constexpr int kBlock = 256;
#ifndef SV_ACC_PREFETCH
#define SV_ACC_PREFETCH 1  // next entry index loaded a step ahead (0: none, 2: next point too -- 162 VGPRs, no gain)
#endif

__device__ __forceinline__ G1Aff load_aff(const G1Aff* __restrict__ a, uint32_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(a + i);
  uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
  G1Aff r;
  r.x.v[0] = q0.x; r.x.v[1] = q0.y; r.x.v[2] = q0.z; r.x.v[3] = q0.w;
  r.x.v[4] = q1.x; r.x.v[5] = q1.y; r.x.v[6] = q1.z; r.x.v[7] = q1.w;
  r.y.v[0] = q2.x; r.y.v[1] = q2.y; r.y.v[2] = q2.z; r.y.v[3] = q2.w;
  r.y.v[4] = q3.x; r.y.v[5] = q3.y; r.y.v[6] = q3.z; r.y.v[7] = q3.w;
  return r;
}

// virtual point idx: P_idx, or phi(P_(idx - nsplit)) = (beta x, y) for a GLV k2 entry (nsplit = n;
// ~0u without GLV): x from the beta-x table, y from the bases
// (phi64: the table holds whole phi(P) records, 64 B, one gather per entry)
__device__ __forceinline__ G1Aff load_vpoint(const G1Aff* __restrict__ bases, const uint4* __restrict__ phix,
                                             uint32_t idx, uint32_t nsplit, int phi64) {
  const bool ph = idx >= nsplit;
  const uint32_t i = ph ? idx - nsplit : idx;
  const uint4* p = reinterpret_cast<const uint4*>(bases + i);
  const uint4* px = ph ? phix + (phi64 ? 4 : 2) * i : p;
  const uint4* py = ph && phi64 ? px : p;
  const uint4 q0 = px[0], q1 = px[1], q2 = py[2], q3 = py[3];
  G1Aff r;
  r.x.v[0] = q0.x; r.x.v[1] = q0.y; r.x.v[2] = q0.z; r.x.v[3] = q0.w;
  r.x.v[4] = q1.x; r.x.v[5] = q1.y; r.x.v[6] = q1.z; r.x.v[7] = q1.w;
  r.y.v[0] = q2.x; r.y.v[1] = q2.y; r.y.v[2] = q2.z; r.y.v[3] = q2.w;
  r.y.v[4] = q3.x; r.y.v[5] = q3.y; r.y.v[6] = q3.z; r.y.v[7] = q3.w;
  return r;
}

__device__ __forceinline__ G1Xyzz load_xyzz(const G1Xyzz* __restrict__ a, uint32_t i) {
  const uint4* p = reinterpret_cast<const uint4*>(a + i);
  G1Xyzz r;
  uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint4 q = p[k];
    d[4 * k + 0] = q.x; d[4 * k + 1] = q.y; d[4 * k + 2] = q.z; d[4 * k + 3] = q.w;
  }
  return r;
}

__device__ __forceinline__ void store_xyzz(G1Xyzz* __restrict__ a, uint32_t i, const G1Xyzz& v) {
  uint4* p = reinterpret_cast<uint4*>(a + i);
  const uint32_t* s = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < 8; k++) p[k] = make_uint4(s[4 * k], s[4 * k + 1], s[4 * k + 2], s[4 * k + 3]);
}

// Bucket-sum records (bsum, pfirst, plast).  The 32-bit chain stores canonical G1Xyzz (128 B).  The
// 29-bit chain (round 6) stores its own state as it is: 4 x 9 limbs, 144 B, X below 8p -- a segment
// end is nine 16-B stores and no conversion (round 4-5 packed the limbs into 8-word x R' values
// after a conditional subtraction of 4p: ~110 VALU instructions in the accumulate's divergent
// segment-end block, i.e. ~70 per bucket entry at 2^20).  The readers convert once per bucket.
// Arrays stay typed G1Xyzz*: rec_at gives record i of either form.
constexpr uint32_t kRec29Words = 4 * r29::L;  // 36
__host__ __device__ __forceinline__ size_t bucket_rec_bytes(int r29) { return r29 ? 4 * kRec29Words : sizeof(G1Xyzz); }
template <class T>
__host__ __device__ __forceinline__ T* rec_at(T* base, size_t i, int r29) {
  using U = typename std::conditional<std::is_const<T>::value, const uint32_t, uint32_t>::type;
  return r29 ? reinterpret_cast<T*>(reinterpret_cast<U*>(base) + kRec29Words * i) : base + i;
}
__device__ __forceinline__ void st_rec29(G1Xyzz* __restrict__ base, size_t i, const r29::Xyzz& a) {
  uint4* o = reinterpret_cast<uint4*>(rec_at(base, i, 1));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
  for (int k = 0; k < 9; k++) o[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}
__device__ __forceinline__ r29::Xyzz ld_rec29(const G1Xyzz* __restrict__ base, size_t i) {
  const uint4* o = reinterpret_cast<const uint4*>(rec_at(base, i, 1));
  r29::Xyzz a;
  uint32_t* w = reinterpret_cast<uint32_t*>(&a);
#pragma unroll
  for (int k = 0; k < 9; k++) {
    const uint4 q = o[k];
    w[4 * k] = q.x, w[4 * k + 1] = q.y, w[4 * k + 2] = q.z, w[4 * k + 3] = q.w;
  }
  return a;
}
// one coordinate (0..3: X, Y, ZZ, ZZZ) of a 29-bit record in field.hpp's canonical x R form
__device__ __forceinline__ Fq rec29_coord_canonical(const G1Xyzz* __restrict__ rec, int c) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(rec) + r29::L * c;
  r29::F f;
#pragma unroll
  for (int i = 0; i < r29::L; i++) f.v[i] = w[i];
  Fq r;
  r29::to_r32(r29::csub<4>(f), r.v);  // X below 8p; the others below 2p (csub leaves them)
  return r;
}
__device__ __forceinline__ void rec29_coord_store(G1Xyzz* __restrict__ rec, int c, const Fq& canon) {
  const r29::F f = r29::to_r29(canon.v);  // below 2p
  uint32_t* w = reinterpret_cast<uint32_t*>(rec) + r29::L * c;
#pragma unroll
  for (int i = 0; i < r29::L; i++) w[i] = f.v[i];
}
__device__ __forceinline__ G1Xyzz load_bucket(const G1Xyzz* __restrict__ a, uint32_t i, int r29w) {
  if (!r29w) return load_xyzz(a, i);
  const G1Xyzz* rec = rec_at(a, i, 1);
  return {rec29_coord_canonical(rec, 0), rec29_coord_canonical(rec, 1), rec29_coord_canonical(rec, 2),
          rec29_coord_canonical(rec, 3)};
}
// store a canonical sum into record i of either form
__device__ __forceinline__ void store_bucket(G1Xyzz* __restrict__ a, uint32_t i, const G1Xyzz& v, int r29w) {
  if (!r29w) {
    store_xyzz(a, i, v);
    return;
  }
  G1Xyzz* rec = rec_at(a, i, 1);
  rec29_coord_store(rec, 0, v.X);
  rec29_coord_store(rec, 1, v.Y);
  rec29_coord_store(rec, 2, v.ZZ);
  rec29_coord_store(rec, 3, v.ZZZ);
}

// ---------------------------------------------------------------------------------------------
__global__ void k_to_mont_bases(const G1Aff* __restrict__ in, G1Aff* __restrict__ out, uint32_t n,
                                uint32_t* __restrict__ err) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1Aff a = load_aff(in, i);
  if (!a.x.is_reduced() || !a.y.is_reduced()) atomicOr(err, 1u);
  G1Aff r;
  if (a.is_identity()) {
    r = a;
  } else {
    r.x = fe_to_mont(a.x);
    r.y = fe_to_mont(a.y);
  }
  reinterpret_cast<uint4*>(out + i)[0] = make_uint4(r.x.v[0], r.x.v[1], r.x.v[2], r.x.v[3]);
  reinterpret_cast<uint4*>(out + i)[1] = make_uint4(r.x.v[4], r.x.v[5], r.x.v[6], r.x.v[7]);
  reinterpret_cast<uint4*>(out + i)[2] = make_uint4(r.y.v[0], r.y.v[1], r.y.v[2], r.y.v[3]);
  reinterpret_cast<uint4*>(out + i)[3] = make_uint4(r.y.v[4], r.y.v[5], r.y.v[6], r.y.v[7]);
}

// Signed windows: digit_w = bits[cw, cw+c) + carry, mapped to (-2^(c-1), 2^(c-1)].  W = ceil(NB/c)
// windows so the top digit never carries out: NB = 255 for full scalars (< r < 2^254), NB = 128 for
// GLV halves (magnitude < 2^127).  f(w, mag, neg) per window.
template <int C, int NB>
__host__ __device__ constexpr int num_windows() { return (NB + C - 1) / C; }
template <int C, int NB = 255, class F>
__device__ __forceinline__ void for_each_digit(const Fr& s, F&& f) {
  constexpr int W = num_windows<C, NB>();
  uint32_t carry = 0;
  const uint32_t half = 1u << (C - 1);
  const uint32_t mask = (1u << C) - 1;
#pragma unroll
  for (int w = 0; w < W; w++) {
    const int pos = w * C;
    const int limb = pos >> 5, off = pos & 31;
    const uint32_t lo = limb < 8 ? s.v[limb] : 0;
    const uint32_t hi = (limb + 1) < 8 ? s.v[limb + 1] : 0;
    uint32_t bits = off ? ((lo >> off) | (hi << (32 - off))) : lo;
    bits = (bits & mask) + carry;
    if (bits > half) {
      // digit = bits - 2^C <= 0; bits == 2^C (all-ones window + carry) is digit 0 with carry 1
      f(w, (1u << C) - bits, 1u);
      carry = 1;
    } else {
      f(w, bits, 0u);
      carry = 0;
    }
  }
}

__device__ __forceinline__ Fr scalar_in(const uint4 q0, const uint4 q1, int mont_in, uint32_t* __restrict__ err) {
  Fr s;
  s.v[0] = q0.x; s.v[1] = q0.y; s.v[2] = q0.z; s.v[3] = q0.w;
  s.v[4] = q1.x; s.v[5] = q1.y; s.v[6] = q1.z; s.v[7] = q1.w;
  if (err && !s.is_reduced()) atomicOr(err, 2u);
  return mont_in ? fe_from_mont(s) : s;
}
__device__ __forceinline__ Fr load_scalar(const Fr* __restrict__ scalars, uint32_t i, int mont_in,
                                          uint32_t* __restrict__ err) {
  const uint4* p = reinterpret_cast<const uint4*>(scalars + i);
  const uint4 q0 = p[0], q1 = p[1];
  Fr s;
  s.v[0] = q0.x; s.v[1] = q0.y; s.v[2] = q0.z; s.v[3] = q0.w;
  s.v[4] = q1.x; s.v[5] = q1.y; s.v[6] = q1.z; s.v[7] = q1.w;
  if (err && !s.is_reduced()) atomicOr(err, 2u);
  return mont_in ? fe_from_mont(s) : s;
}

// Entries of real point i for the sort passes.  Without GLV: the W signed digits of its scalar,
// all for virtual point i (half 0).  With GLV the scalar is split here (glv.hpp; the halves
// are stored for the scatter pass on the device path, see store()): the W digits of k1 belong to virtual point i (P_i, half 0) and the W digits of k2 to
// virtual point n + i (phi(P_i), half 1), each half's sign folded into its digits' signs; both
// halves share the W windows' buckets.  f(w, mag, neg, half) per digit.
template <int C, bool GLV>
struct Digits {
  static constexpr int NB = GLV ? 128 : 255;
  static constexpr int W = num_windows<C, NB>();
  static constexpr int EP = GLV ? 2 * W : W;  // entries per real point
  uint32_t h[GLV ? 2 : 1][GLV ? 4 : 8];
  uint32_t sgn[GLV ? 2 : 1];
  __device__ __forceinline__ void load(const Fr* __restrict__ scalars, uint32_t i, int mont_in,
                                       uint32_t* __restrict__ err) {
    from(load_scalar(scalars, i, mont_in, err));
  }
  __device__ __forceinline__ void from(const Fr& s) {
    if constexpr (GLV) {
      uint32_t h1[4], h2[4];
      glv_split(s.v, h1, h2);
#pragma unroll
      for (int k = 0; k < 4; k++) h[0][k] = h1[k], h[1][k] = h2[k];
#pragma unroll
      for (int q = 0; q < 2; q++) {
        sgn[q] = h[q][3] >> 31;
        h[q][3] &= 0x7fffffffu;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 8; k++) h[0][k] = s.v[k];
      sgn[0] = 0;
    }
  }
  // The histogram pass stores what load() derived (GLV: both halves, the sign in bit 31 of the top
  // word; else the canonical scalar): 32 B per point, so the scatter pass reads it back instead of
  // converting from Montgomery form and splitting again (SVGPU_SORT_HALVES=0: recompute, as before)
  __device__ __forceinline__ void store(uint4* __restrict__ hv, uint32_t i) const {
    if constexpr (GLV) {
      hv[2 * i] = make_uint4(h[0][0], h[0][1], h[0][2], h[0][3] | (sgn[0] << 31));
      hv[2 * i + 1] = make_uint4(h[1][0], h[1][1], h[1][2], h[1][3] | (sgn[1] << 31));
    } else {
      hv[2 * i] = make_uint4(h[0][0], h[0][1], h[0][2], h[0][3]);
      hv[2 * i + 1] = make_uint4(h[0][4], h[0][5], h[0][6], h[0][7]);
    }
  }
  __device__ __forceinline__ void load_stored(const uint4* __restrict__ hv, uint32_t i) {
    const uint4 a = hv[2 * i], b = hv[2 * i + 1];
    if constexpr (GLV) {
      h[0][0] = a.x; h[0][1] = a.y; h[0][2] = a.z; h[0][3] = a.w & 0x7fffffffu;
      h[1][0] = b.x; h[1][1] = b.y; h[1][2] = b.z; h[1][3] = b.w & 0x7fffffffu;
      sgn[0] = a.w >> 31;
      sgn[1] = b.w >> 31;
    } else {
      h[0][0] = a.x; h[0][1] = a.y; h[0][2] = a.z; h[0][3] = a.w;
      h[0][4] = b.x; h[0][5] = b.y; h[0][6] = b.z; h[0][7] = b.w;
      sgn[0] = 0;
    }
  }
  template <class F>
  __device__ __forceinline__ void each(F&& f) const {
#pragma unroll
    for (int q = 0; q < (GLV ? 2 : 1); q++) {
      Fr s;
      if constexpr (GLV) {
#pragma unroll
        for (int k = 0; k < 4; k++) s.v[k] = h[q][k], s.v[4 + k] = 0u;
      } else {
#pragma unroll
        for (int k = 0; k < 8; k++) s.v[k] = h[0][k];
      }
      const uint32_t sg = sgn[q];
      for_each_digit<C, NB>(s, [&](int w, uint32_t mag, uint32_t neg) { f(w, mag, neg ^ sg, (uint32_t)q); });
    }
  }
};

// GLV: phi(P_i) = (beta x_i, y_i); only beta x_i is stored (phix[i], 32 B, written by k_bin_hist),
// the accumulate reads y_i from the bases (identity (0, 0) maps to itself).  With err set the point's
// coordinates are checked to be reduced (Montgomery input is used as is by the 2p-domain adds).
__device__ __forceinline__ void glv_phix(const G1Aff* __restrict__ bases, uint32_t i, uint4* __restrict__ phix,
                                         int phi64, uint32_t* __restrict__ err) {
  const uint4* b = reinterpret_cast<const uint4*>(bases + i);
  Fq x, beta;
  const uint4 x0 = b[0], x1 = b[1];
  x.v[0] = x0.x; x.v[1] = x0.y; x.v[2] = x0.z; x.v[3] = x0.w;
  x.v[4] = x1.x; x.v[5] = x1.y; x.v[6] = x1.z; x.v[7] = x1.w;
#pragma unroll
  for (int j = 0; j < 8; j++) beta.v[j] = GLV_BETA_MONT[j];
  const Fq bx = x * beta;
  uint4* o = phix + (phi64 ? 4 : 2) * i;
  o[0] = make_uint4(bx.v[0], bx.v[1], bx.v[2], bx.v[3]);
  o[1] = make_uint4(bx.v[4], bx.v[5], bx.v[6], bx.v[7]);
  if (phi64 || err) {
    const uint4 y0 = b[2], y1 = b[3];
    if (phi64) {
      o[2] = y0;
      o[3] = y1;
    }
    if (err) {
      Fq y;
      y.v[0] = y0.x; y.v[1] = y0.y; y.v[2] = y0.z; y.v[3] = y0.w;
      y.v[4] = y1.x; y.v[5] = y1.y; y.v[6] = y1.z; y.v[7] = y1.w;
      if (!x.is_reduced() || !y.is_reduced()) atomicOr(err, 1u);
    }
  }
}

// Host-fed pieces: the piece's table once its bases have landed (its sort ran on the scalars alone)
__global__ void k_glv_phix(const G1Aff* __restrict__ bases, uint32_t n, uint4* __restrict__ phix, int phi64,
                           uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) glv_phix(bases, i, phix, phi64, err);
}

// The 29-bit chain's table of virtual points (p.r29, replaces phix): every record the chain's own
// limbs, x R' as 9 x 29-bit limbs for x then y (72 B, 9 uint2), so the accumulate's per-entry point
// load is the whole conversion -- converted once per point here instead of once per bucket entry
// (16 entries per point at 2^20).  Round 6: the limbs themselves (round 4-5 stored 8-word x R'
// values, 64 B, and split them into limbs per entry: ~35 VALU instructions per entry).  P_i at
// record i and, with GLV, phi(P_i) = (beta x_i, y_i) at record nsplit + i.  With err set the bases
// are checked to be reduced (Montgomery input is used as is).
static constexpr int kPhiVtab = 2;  // k_bin_hist's phi64 value for "phix is the r29 table"
static constexpr int kVtabRec = 9;  // uint2 per record
__device__ __forceinline__ void st_rec29(uint2* o, const r29::F& x, const r29::F& y) {
  o[0] = make_uint2(x.v[0], x.v[1]);
  o[1] = make_uint2(x.v[2], x.v[3]);
  o[2] = make_uint2(x.v[4], x.v[5]);
  o[3] = make_uint2(x.v[6], x.v[7]);
  o[4] = make_uint2(x.v[8], y.v[0]);
  o[5] = make_uint2(y.v[1], y.v[2]);
  o[6] = make_uint2(y.v[3], y.v[4]);
  o[7] = make_uint2(y.v[5], y.v[6]);
  o[8] = make_uint2(y.v[7], y.v[8]);
}
__device__ __forceinline__ void ld_rec29(const uint2* __restrict__ o, r29::F& x, r29::F& y) {
  uint2 q[kVtabRec];
#pragma unroll
  for (int k = 0; k < kVtabRec; k++) q[k] = o[k];
  x.v[0] = q[0].x, x.v[1] = q[0].y, x.v[2] = q[1].x, x.v[3] = q[1].y, x.v[4] = q[2].x, x.v[5] = q[2].y;
  x.v[6] = q[3].x, x.v[7] = q[3].y, x.v[8] = q[4].x;
  y.v[0] = q[4].y, y.v[1] = q[5].x, y.v[2] = q[5].y, y.v[3] = q[6].x, y.v[4] = q[6].y, y.v[5] = q[7].x;
  y.v[6] = q[7].y, y.v[7] = q[8].x, y.v[8] = q[8].y;
}
// uint4 per point of the r29 table (its buffer is carved in uint4): GLV two 72-B records, else one
// (padded to 80 B per point so host-fed pieces' table slices stay uint4-aligned)
__host__ __device__ constexpr size_t vtab_uint4_per_point(bool glv) { return glv ? 9 : 5; }
__device__ __forceinline__ void vtab_put_pt(const G1Aff& a, uint32_t i, uint4* __restrict__ vtab, uint32_t nsplit,
                                            bool glv, uint32_t* __restrict__ err) {
  if (err && (!a.x.is_reduced() || !a.y.is_reduced())) atomicOr(err, 1u);
  const r29::F y = r29::to_r29(a.y.v), x = r29::to_r29(a.x.v);  // below 2p
  uint2* t = reinterpret_cast<uint2*>(vtab);
  st_rec29(t + kVtabRec * (size_t)i, x, y);
  if (glv) {  // beta x in the 29-bit form directly: beta R' (GLV_BETA_MONT re-expressed, 2^261)
    constexpr uint32_t kBeta29[r29::L] = {0xa337995u, 0x158d1d23u, 0x189c9b98u, 0x12fa4e45u, 0x185faadcu,
                                         0x176f16du, 0xeed93bau,  0x14291140u, 0xc0afeu};
    r29::F beta;
#pragma unroll
    for (int j = 0; j < r29::L; j++) beta.v[j] = kBeta29[j];
    st_rec29(t + kVtabRec * ((size_t)nsplit + i), r29::mul(x, beta), y);  // below 2p
  }
}
__device__ __forceinline__ void vtab_put(const G1Aff* __restrict__ bases, uint32_t i, uint4* __restrict__ vtab,
                                         uint32_t nsplit, bool glv, uint32_t* __restrict__ err) {
  vtab_put_pt(load_aff(bases, i), i, vtab, nsplit, glv, err);
}
// Host-fed pieces with the 29-bit chain: the piece's table once its bases have landed
__global__ void k_vtab(const G1Aff* __restrict__ bases, uint32_t n, uint4* __restrict__ vtab, int glv,
                       uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) vtab_put(bases, i, vtab, n, glv != 0, err);
}

// Montgomery-form bases that no other pass reads before the accumulate (no GLV table, host-fed)
__global__ void k_check_bases(const G1Aff* __restrict__ bases, uint32_t n, uint32_t* __restrict__ err) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1Aff a = load_aff(bases, i);
  if (!a.x.is_reduced() || !a.y.is_reduced()) atomicOr(err, 1u);
}

// ---- two-level counting sort of the n * W (point, digit) entries by bucket ------------------
// Bucket b = |digit| - 1 of window w splits into a coarse bin b >> FB (NBIN = 2^CB bins per window)
// and a fine index b & (2^FB - 1).  Pass 1 (k_bin_hist): per block of sort_chunk(c) points, every
// window's digits, LDS histogram of (window, bin).  Pass 2 (k_bin_scan_chunks, k_bin_scan): global
// offsets of every (window, bin, block) run.  Pass 3 (k_bin_scatter): the digits again (from the halves pass 1 stored), each
// entry appended to its block's run -> tmp (u64: fine << 32 | point | sign << 31); a block's runs
// are short contiguous spans, so writes merge in L2.  Pass 4 (k_fine_sort): one block per
// (window, bin) counting-sorts its ~n / NBIN entries by fine index inside that bin's region (L2
// resident), writes ent[], the global bucket offsets gst[] and the owner bucket tstart[t] of every
// accumulate chunk [tK, tK + K).  No per-(window, point) digit array is ever stored.
// points per block in passes 1 and 3: sort_chunk (below), 256 when the LDS staging of W digits per
// point would not fit (small c, many windows)
// Points per block of the histogram / scatter passes (ep: entries per point).  1024 (round 3) halves
// the block count, so each (window, bin) run a scatter block writes is ~16 entries (64 B) instead of
// ~8: sort 0.221 -> 0.206 ms at 2^20.  LDS: the scatter stages CH * ep u32 entries (2048 spilled
// the scatter's digit registers: 336 B scratch, one wave per SIMD).
#ifndef SV_SORT_CHUNK
#define SV_SORT_CHUNK 1024
#endif
__host__ __device__ constexpr uint32_t sort_chunk(int ep) {
  return ep > 20 ? 256u : (ep > 16 && SV_SORT_CHUNK > 1024 ? 1024u : (uint32_t)SV_SORT_CHUNK);
}
// coarse bits: 2^CB bins per window, so that W * 2^CB ~ 1024 fine-sort regions of ~16K entries at
// 2^20 (LDS-staged in k_fine_sort) -- 64 bins for the 16 full-width windows, 128 for the 8 GLV ones
__host__ __device__ constexpr int coarse_bits(int c, int nb) { return c - 1 < (nb == 128 ? 7 : 6) ? c - 1 : (nb == 128 ? 7 : 6); }
__host__ __device__ constexpr int ceil_log2(int x) { return x <= 1 ? 0 : 1 + ceil_log2((x + 1) / 2); }

// exclusive scan of x[0 .. N) in LDS by a 256-thread block (N <= 4096); returns the total
template <int N>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t* x, uint32_t* part) {
  constexpr int PER = (N + kBlock - 1) / kBlock;
  const int tid = threadIdx.x;
  uint32_t loc[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int k = tid * PER + j;
    loc[j] = k < N ? x[k] : 0u;
    sum += loc[j];
  }
  part[tid] = sum;
  __syncthreads();
  for (int off = 1; off < kBlock; off <<= 1) {
    const uint32_t u = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += u;
    __syncthreads();
  }
  uint32_t run = part[tid] - sum;
  const uint32_t total = part[kBlock - 1];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const int k = tid * PER + j;
    if (k < N) x[k] = run;
    run += loc[j];
  }
  __syncthreads();
  return total;
}

// Coarse-binned entries (tmp[]): u64 fine << 32 | point | sign << 31, or -- when the virtual
// point index fits in 31 - FB bits (every size up to 2^22 points) -- packed into u32 as
// fine << (32 - FB) | sign << (31 - FB) | point, which halves the scatter's writes and the fine
// sort's reads.  The fine sort expands either form to the u64 layout in registers.
__device__ __forceinline__ uint32_t pack_entry32(uint32_t fine, uint32_t neg, uint32_t pt, uint32_t fb) {
  return (fb ? fine << (32 - fb) : 0u) | (neg << (31 - fb)) | pt;
}
__device__ __forceinline__ uint64_t load_entry(const uint64_t* __restrict__ tmp, uint32_t i, int e32, uint32_t fb) {
  if (!e32) return tmp[i];
  const uint32_t v = reinterpret_cast<const uint32_t*>(tmp)[i];
  const uint32_t fine = fb ? v >> (32 - fb) : 0u, neg = (v >> (31 - fb)) & 1u, pt = v & ((1u << (31 - fb)) - 1u);
  return ((uint64_t)fine << 32) | pt | (neg << 31);
}

// Logical block of the histogram / scatter passes.  Workgroups are dispatched round-robin over the
// 8 XCDs, so consecutive blocks sit on different L2s; both passes store per-block counts column-wise
// (bcnt[key * nblk + blk], 32 blocks per 128-B line) and runs of consecutive blocks side by side in
// tmp, and a line filled from 8 L2s is written back 8 times, partially.  xcd != 0 gives each XCD a
// contiguous range of logical blocks instead (a bijection; the tail n % 8 blocks keep their index).
__device__ __forceinline__ uint32_t sort_block(uint32_t b, uint32_t n, int xcd) {
  const uint32_t nfull = n & ~7u;
  if (!xcd || b >= nfull) return b;
  return (b & 7u) * (nfull >> 3) + (b >> 3);
}

// With GLV the pass also writes the beta-x table of its points (phix, see glv_phix).
template <int C, bool GLV>
__global__ void __launch_bounds__(kBlock) k_bin_hist(const Fr* __restrict__ scalars, uint32_t n, int mont_in,
                                                     uint32_t nblk, uint32_t* __restrict__ bcnt,
                                                     uint32_t* __restrict__ err, const G1Aff* __restrict__ bases,
                                                     uint4* __restrict__ phix, int phi64, int check_bases,
                                                     int xcd, int bm, uint32_t w0, uint32_t nw,
                                                     uint4* __restrict__ stored, int pf) {
  using D = Digits<C, GLV>;
  constexpr int W = D::W, LOGB = C - 1;
  constexpr int CB = coarse_bits(C, D::NB), FB = LOGB - CB, NBIN = 1 << CB;
  // windows [w0, w0 + nw) only (the MSM's window halves are sorted separately, see msm_run_impl):
  // keys (w - w0) * NBIN + bin
  const uint32_t nk = nw * NBIN;
  __shared__ uint32_t h[W * NBIN];
  for (int k = threadIdx.x; k < W * NBIN; k += kBlock) h[k] = 0;
  __syncthreads();
  constexpr uint32_t CH = sort_chunk(D::EP);
  const uint32_t blk = sort_block(blockIdx.x, gridDim.x, xcd);
  const uint32_t lo = blk * CH, hi = min(n, lo + CH);
  auto count = [&](const D& d) {
    d.each([&](int w, uint32_t mag, uint32_t, uint32_t) {
      if (mag && (uint32_t)w - w0 < nw) atomicAdd(&h[(w - w0) * NBIN + ((mag - 1) >> FB)], 1u);
    });
  };
  if (phix && phi64 == kPhiVtab && pf) {
    // Round 6: the 29-bit table path with the next point's scalar and base loaded one iteration
    // ahead (the pass is load-latency-bound: ~4 dependent iterations per thread at 4 waves/SIMD)
    uint32_t i = lo + threadIdx.x;
    const uint4* sp = reinterpret_cast<const uint4*>(scalars);
    const uint4* bp = reinterpret_cast<const uint4*>(bases);
    uint4 s0{}, s1{}, b0{}, b1{}, b2{}, b3{};
    if (i < hi) {
      s0 = sp[2 * (size_t)i], s1 = sp[2 * (size_t)i + 1];
      b0 = bp[4 * (size_t)i], b1 = bp[4 * (size_t)i + 1], b2 = bp[4 * (size_t)i + 2], b3 = bp[4 * (size_t)i + 3];
    }
    for (; i < hi; i += kBlock) {
      G1Aff a;
      a.x.v[0] = b0.x; a.x.v[1] = b0.y; a.x.v[2] = b0.z; a.x.v[3] = b0.w;
      a.x.v[4] = b1.x; a.x.v[5] = b1.y; a.x.v[6] = b1.z; a.x.v[7] = b1.w;
      a.y.v[0] = b2.x; a.y.v[1] = b2.y; a.y.v[2] = b2.z; a.y.v[3] = b2.w;
      a.y.v[4] = b3.x; a.y.v[5] = b3.y; a.y.v[6] = b3.z; a.y.v[7] = b3.w;
      const uint4 c0 = s0, c1 = s1;
      const uint32_t j = i + kBlock;
      if (j < hi) {
        s0 = sp[2 * (size_t)j], s1 = sp[2 * (size_t)j + 1];
        b0 = bp[4 * (size_t)j], b1 = bp[4 * (size_t)j + 1], b2 = bp[4 * (size_t)j + 2], b3 = bp[4 * (size_t)j + 3];
      }
      vtab_put_pt(a, i, phix, n, GLV, check_bases ? err : nullptr);
      D d;
      d.from(scalar_in(c0, c1, mont_in, err));
      if (stored) d.store(stored, i);
      count(d);
    }
  } else
  for (uint32_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    // Montgomery bases are checked here (canonical ones by k_to_mont_bases)
    if (phix && phi64 == kPhiVtab) {  // the 29-bit chain's table (n = nsplit on the device path)
      vtab_put(bases, i, phix, n, GLV, check_bases ? err : nullptr);
    } else if constexpr (GLV) {
      if (phix) glv_phix(bases, i, phix, phi64, check_bases ? err : nullptr);  // (null: bases not landed yet, k_glv_phix later)
    } else {
      if (check_bases) {
        const G1Aff a = load_aff(bases, i);
        if (!a.x.is_reduced() || !a.y.is_reduced()) atomicOr(err, 1u);
      }
    }
    D d;
    d.load(scalars, i, mont_in, err);
    if (stored) d.store(stored, i);
    count(d);
  }
  __syncthreads();
  // bm: block-major bcnt[blk * nk + key], one contiguous row per block (the scan reads it in
  // 32-key tiles); else key-major bcnt[key * nblk + blk] (round 2)
  for (uint32_t k = threadIdx.x; k < nk; k += kBlock)
    bcnt[bm ? (size_t)blk * nk + k : (size_t)k * nblk + blk] = h[k];
}

// one 256-thread block per (window, bin): exclusive scan over blocks in place, total -> btot
__global__ void __launch_bounds__(kBlock) k_bin_scan_chunks(uint32_t* __restrict__ bcnt, uint32_t nblk,
                                                            uint32_t* __restrict__ btot) {
  __shared__ uint32_t part[kBlock];
  uint32_t* c = bcnt + (size_t)blockIdx.x * nblk;
  const uint32_t tid = threadIdx.x, per = (nblk + kBlock - 1) / kBlock;
  const uint32_t lo = min(nblk, tid * per), hi = min(nblk, lo + per);
  uint32_t sum = 0;
  for (uint32_t b = lo; b < hi; b++) sum += c[b];
  part[tid] = sum;
  __syncthreads();
  for (uint32_t off = 1; off < kBlock; off <<= 1) {
    const uint32_t u = tid >= off ? part[tid - off] : 0u;
    __syncthreads();
    part[tid] += u;
    __syncthreads();
  }
  uint32_t run = part[tid] - sum;
  for (uint32_t b = lo; b < hi; b++) {
    const uint32_t v = c[b];
    c[b] = run;
    run += v;
  }
  if (tid == kBlock - 1) btot[blockIdx.x] = part[kBlock - 1];
}

// Block-major counts (bcnt[blk * nk + key]): one 1024-thread block per 32 keys.  Thread (grp, kk)
// walks rows grp * per .. of key 32 tile + kk, so each row access of a wave reads or writes two whole
// 128-B lines; exclusive scan over blocks in place, total -> btot.
template <int KT>  // keys per tile (32 or 16): 1024 / KT row groups per block
__global__ void __launch_bounds__(1024) k_bin_scan_tiles(uint32_t* __restrict__ bcnt, uint32_t nblk, uint32_t nk,
                                                         uint32_t* __restrict__ btot) {
  constexpr int G = 1024 / KT;
  __shared__ uint32_t part[G][KT + 1];
  const uint32_t kk = threadIdx.x % KT, grp = threadIdx.x / KT, key = blockIdx.x * KT + kk;
  const uint32_t per = (nblk + G - 1) / G, lo = min(nblk, grp * per), hi = min(nblk, lo + per);
  const bool live = key < nk;
  uint32_t* c = bcnt + key;
  uint32_t sum = 0;
  if (live) {
#pragma unroll 8
    for (uint32_t b = lo; b < hi; b++) sum += c[(size_t)b * nk];
  }
  part[grp][kk] = sum;
  __syncthreads();
  if (threadIdx.x < KT) {  // per key: exclusive scan over the G row groups
    uint32_t run = 0;
    for (int g = 0; g < G; g++) {
      const uint32_t v = part[g][threadIdx.x];
      part[g][threadIdx.x] = run;
      run += v;
    }
    if (blockIdx.x * KT + threadIdx.x < nk) btot[blockIdx.x * KT + threadIdx.x] = run;
  }
  __syncthreads();
  if (live) {
    uint32_t run = part[grp][kk];
#pragma unroll 8
    for (uint32_t b = lo; b < hi; b++) {
      const uint32_t v = c[(size_t)b * nk];
      c[(size_t)b * nk] = run;
      run += v;
    }
  }
}

// one 1024-thread block: exclusive scan of btot over all (window, bin) -> bstart; bstart[nwb] = total
__global__ void __launch_bounds__(1024) k_bin_scan(const uint32_t* __restrict__ btot, uint32_t nwb,
                                                   uint32_t* __restrict__ bstart, uint32_t* __restrict__ gst_end) {
  __shared__ uint32_t part[1024];
  const uint32_t tid = threadIdx.x;
  const uint32_t per = (nwb + 1023) / 1024;
  const uint32_t lo = min(nwb, tid * per), hi = min(nwb, lo + per);
  uint32_t s = 0;
  for (uint32_t k = lo; k < hi; k++) s += btot[k];
  part[tid] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint32_t v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  uint32_t run = part[tid] - s;
  for (uint32_t k = lo; k < hi; k++) {
    bstart[k] = run;
    run += btot[k];
  }
  if (tid == 1023) {
    bstart[nwb] = part[1023];
    *gst_end = part[1023];  // gst[nbt]: the entry total (k_fine_sort writes the other bucket starts)
  }
}

// Pass 3: the block's entries are first placed in LDS grouped by (window, bin), then each group
// is copied to its global run with consecutive lanes writing consecutive addresses.  Entry point
// index: the virtual point (i, or n + i for a GLV k2 digit).  The block's own (window, bin) counts
// are not recounted: they are the differences of consecutive block offsets that k_bin_scan_chunks
// left in bcnt (btot for the last block), which halves the LDS atomics of the pass.
template <int C, bool GLV>
__global__ void __launch_bounds__(kBlock) k_bin_scatter(const Fr* __restrict__ scalars, uint32_t n, int mont_in,
                                                        uint32_t nblk, const uint32_t* __restrict__ bcnt,
                                                        const uint32_t* __restrict__ btot,
                                                        const uint32_t* __restrict__ bstart,
                                                        uint64_t* __restrict__ tmp, int e32, int xcd, int bm,
                                                        uint32_t w0, uint32_t nw, const uint4* __restrict__ stored) {
  using D = Digits<C, GLV>;
  constexpr int W = D::W, LOGB = C - 1;
  constexpr int CB = coarse_bits(C, D::NB), FB = LOGB - CB, NBIN = 1 << CB, NK = W * NBIN;
  const uint32_t nk = nw * NBIN;  // keys of windows [w0, w0 + nw), (w - w0) * NBIN + bin
  // staged entry: local point (LP bits) | half << LP | sign << (LP + 1) | fine << (LP + 2) | (window, bin) key << (LP + 2 + FB)
  constexpr int LP = ceil_log2((int)sort_chunk(D::EP));
  static_assert(LP + 2 + FB + ceil_log2(NK) <= 32, "staged entry overflows 32 bits");
  constexpr uint32_t FMASK = (1u << FB) - 1;
  constexpr uint32_t CH = sort_chunk(D::EP), PT = CH / kBlock;
  __shared__ uint32_t off[NK];   // local group offsets
  __shared__ uint32_t cur[NK];   // cursors
  __shared__ uint32_t part[kBlock];
  __shared__ uint32_t stage[CH * D::EP];  // see the layout above (no separate key array: 3 blocks per CU)
  const uint32_t blk = sort_block(blockIdx.x, gridDim.x, xcd), lo = blk * CH, hi = min(n, lo + CH);
  for (uint32_t k = threadIdx.x; k < NK; k += kBlock) {
    if (k >= nk) {
      off[k] = 0;
      continue;
    }
    const size_t at = bm ? (size_t)blk * nk + k : (size_t)k * nblk + blk;
    off[k] = (blk + 1 < nblk ? bcnt[bm ? at + nk : at + 1] : btot[k]) - bcnt[at];
  }
  D dg[PT];
#pragma unroll
  for (int j = 0; j < (int)PT; j++) {
    const uint32_t i = lo + threadIdx.x + j * kBlock;
    if (i < hi) {
      if (stored) dg[j].load_stored(stored, i);  // written by this sort's k_bin_hist
      else dg[j].load(scalars, i, mont_in, nullptr);
    }
  }
  __syncthreads();
  const uint32_t total = block_excl_scan<NK>(off, part);
  for (int k = threadIdx.x; k < NK; k += kBlock) cur[k] = off[k];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < (int)PT; j++) {
    const uint32_t li = threadIdx.x + j * kBlock;
    if (lo + li < hi) {
      dg[j].each([&](int w, uint32_t mag, uint32_t neg, uint32_t half) {
        if (mag && (uint32_t)w - w0 < nw) {
          const uint32_t b = mag - 1;
          const uint32_t k = (w - w0) * NBIN + (b >> FB);
          const uint32_t pos = atomicAdd(&cur[k], 1u);
          stage[pos] = li | (half << LP) | (neg << (LP + 1)) | ((b & FMASK) << (LP + 2)) | (k << (LP + 2 + FB));
        }
      });
    }
  }
  __syncthreads();
  // global position of local slot x = gbase[key] + x  (cur[] reused for gbase)
  for (uint32_t k = threadIdx.x; k < nk; k += kBlock)
    cur[k] = bstart[k] + bcnt[bm ? (size_t)blk * nk + k : (size_t)k * nblk + blk] - off[k];
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < total; x += kBlock) {
    const uint32_t e = stage[x];
    const uint32_t pt = lo + (e & ((1u << LP) - 1u)) + (((e >> LP) & 1u) ? n : 0u);
    const uint32_t dst = cur[e >> (LP + 2 + FB)] + x, fine = (e >> (LP + 2)) & FMASK, neg = (e >> (LP + 1)) & 1u;
    if (e32) reinterpret_cast<uint32_t*>(tmp)[dst] = pack_entry32(fine, neg, pt, FB);
    else tmp[dst] = ((uint64_t)fine << 32) | pt | (neg << 31);
  }
}

// one block per (window, bin): counting sort by the fine index within the bin's region.
// Regions of up to kFineCap entries (every bin but the short top window's at n = 2^20) are read
// from tmp ONCE into registers and sorted into an LDS copy of the region, which is then written to
// ent[] with consecutive lanes on consecutive addresses: the direct scatter of 4-byte entries to
// global memory cost ~5x its bytes in partial-line write traffic (PMC WRITE_SIZE, r01).  Larger
// regions are processed in LDS chunks of the same size (below); the two cases are separate
// instantiations (BIG), each block leaving at once unless its region is of its kind, so the staged
// one keeps to <= 64 VGPRs (two 1024-thread blocks per CU).
static constexpr uint32_t kFineR = 18;                 // entries per thread held in registers
static constexpr uint32_t kFineCap = 1024 * kFineR;    // region entries staged in LDS
static constexpr uint32_t kChunkR = 12, kChunk = 1024 * kChunkR;  // large regions: LDS chunk
static constexpr size_t kFineLds = (512 + 1024 + (size_t)kFineCap) * 4;  // 78 KiB: 2 blocks per CU
// MODE 0: staged regions only, 1: large regions only, 2 (round 3, default): both kinds in ONE launch,
// blocks in reverse (window, bin) order -- the crowded regions are the top window's, and as the
// launch's first blocks they run beside the small regions instead of as a separate serial launch
// (two launches: 37 + 35 us at 2^20, the large one a tail of a few dozen long blocks).
// one region (window, bin) = wb: staged in LDS whole (STAGED) or in chunks
template <bool STAGED>
__device__ __forceinline__ void fine_region(const uint64_t* __restrict__ tmp, int e32, uint32_t wb, uint32_t s0,
                                            uint32_t s1, uint32_t FB, uint32_t K, uint32_t* __restrict__ gst,
                                            uint32_t* __restrict__ tstart, uint32_t* __restrict__ ent,
                                            uint32_t* fine_lds) {
  uint32_t* fc = fine_lds;           // [512] fine-bucket counters / cursors
  uint32_t* part = fine_lds + 512;   // [1024] scan partials
  uint32_t* out = fine_lds + 1536;   // [kFineCap] the sorted region
  const uint32_t tid = threadIdx.x, NF = 1u << FB, len = s1 - s0;
  for (uint32_t f = tid; f < NF; f += 1024) fc[f] = 0;
  __syncthreads();
  uint64_t x[kFineR];
  if constexpr (STAGED) {
#pragma unroll
    for (uint32_t r = 0; r < kFineR; r++) {
      const uint32_t i = tid + r * 1024;
      x[r] = i < len ? load_entry(tmp, s0 + i, e32, FB) : 0;
    }
#pragma unroll
    for (uint32_t r = 0; r < kFineR; r++)
      if (tid + r * 1024 < len) atomicAdd(&fc[(uint32_t)(x[r] >> 32)], 1u);
  } else {
    uint32_t e = s0 + tid;
    for (; e + 3 * 1024 < s1; e += 4 * 1024) {  // 4 loads in flight per thread
      const uint32_t f0 = (uint32_t)(load_entry(tmp, e, e32, FB) >> 32);
      const uint32_t f1 = (uint32_t)(load_entry(tmp, e + 1024, e32, FB) >> 32);
      const uint32_t f2 = (uint32_t)(load_entry(tmp, e + 2048, e32, FB) >> 32);
      const uint32_t f3 = (uint32_t)(load_entry(tmp, e + 3072, e32, FB) >> 32);
      atomicAdd(&fc[f0], 1u);
      atomicAdd(&fc[f1], 1u);
      atomicAdd(&fc[f2], 1u);
      atomicAdd(&fc[f3], 1u);
    }
    for (; e < s1; e += 1024) atomicAdd(&fc[(uint32_t)(load_entry(tmp, e, e32, FB) >> 32)], 1u);
  }
  __syncthreads();
  // exclusive scan of fc[0 .. NF) (NF <= 512)
  const uint32_t v = tid < NF ? fc[tid] : 0;
  part[tid] = v;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint32_t u = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += u;
    __syncthreads();
  }
  if (tid < NF) {
    const uint32_t st = s0 + part[tid] - v, en = st + v;
    const uint32_t g = wb * NF + tid;  // global bucket = w * B + b
    gst[g] = st;
    fc[tid] = STAGED ? st - s0 : st;
    for (uint32_t t = (st + K - 1) / K; t * K < en; t++) tstart[t] = g;
  }
  __syncthreads();
  if constexpr (STAGED) {
#pragma unroll
    for (uint32_t r = 0; r < kFineR; r++)
      if (tid + r * 1024 < len) out[atomicAdd(&fc[(uint32_t)(x[r] >> 32)], 1u)] = (uint32_t)x[r];
    __syncthreads();
    for (uint32_t i = tid; i < len; i += 1024) ent[s0 + i] = out[i];
    return;
  }
  // Large region: chunks of kChunk entries (12 per thread: the instantiation stays <= 64 VGPRs), each counting-sorted in LDS (chunk-local counts lc,
  // starts ls) and written as one contiguous run per fine bucket at that bucket's global cursor fc.
  uint32_t* lc = part;  // chunk counts reuse the scan buffer's first 512 words ...
  uint32_t* ls = part + 512;  // ... and chunk-local starts its second half
  for (uint32_t c0 = s0; c0 < s1; c0 += kChunk) {
    const uint32_t clen = min(kChunk, s1 - c0);
    if (tid < NF) lc[tid] = 0;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kChunkR; r++) {
      const uint32_t i = tid + r * 1024;
      x[r] = i < clen ? load_entry(tmp, c0 + i, e32, FB) : 0;
      if (i < clen) atomicAdd(&lc[(uint32_t)(x[r] >> 32)], 1u);
    }
    __syncthreads();
    // exclusive scan of lc[0 .. NF) by one wave per 64 buckets + a serial pass over the 8 totals
    if (tid < NF) {
      uint32_t v2 = lc[tid], incl = v2;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o);
        if ((tid & 63) >= (uint32_t)o) incl += u;
      }
      ls[tid] = incl - v2;  // exclusive within the wave
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t run = 0;
      for (uint32_t w = 0; w < NF; w += 64) {
        const uint32_t last = min(NF, w + 64) - 1;
        const uint32_t tot = ls[last] + lc[last];
        out[kFineCap - 8 + (w >> 6)] = run;  // per-wave offsets parked at the end of out[]
        run += tot;
      }
    }
    __syncthreads();
    uint32_t base_f = 0;
    if (tid < NF) base_f = ls[tid] + out[kFineCap - 8 + (tid >> 6)];
    __syncthreads();
    if (tid < NF) {
      ls[tid] = base_f;
      lc[tid] = base_f;  // lc becomes the chunk-local cursor
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kChunkR; r++)
      if (tid + r * 1024 < clen) out[atomicAdd(&lc[(uint32_t)(x[r] >> 32)], 1u)] = (uint32_t)x[r];
    __syncthreads();
    // 16 lanes per fine bucket run (a chunk holds ~kChunk / NF ~ 24 entries per bucket):
    // out[ls[f] .. lc[f]) -> ent[fc[f] ..), consecutive lanes on consecutive addresses
    for (uint32_t f = tid >> 4; f < NF; f += 64) {
      const uint32_t st = ls[f], cnt = lc[f] - st, dst = fc[f];
      for (uint32_t j = tid & 15; j < cnt; j += 16) ent[dst + j] = out[st + j];
    }
    __syncthreads();
    if (tid < NF) fc[tid] += lc[tid] - ls[tid];
    __syncthreads();
  }
}


// MODE 0: staged regions only, 1: large regions only, 2 (round 3, default): both kinds in ONE launch,
// blocks in reverse (window, bin) order -- the crowded regions are the top window's, and as the
// launch's first blocks they run beside the small regions instead of as a separate serial launch
// (two launches: 37 + 35 us at 2^20, the large one a tail of a few dozen long blocks).
template <int MODE>
__global__ void __launch_bounds__(1024) k_fine_sort(const uint64_t* __restrict__ tmp, int e32,
                                                    const uint32_t* __restrict__ bstart, uint32_t FB, uint32_t K,
                                                    uint32_t* __restrict__ gst, uint32_t* __restrict__ tstart,
                                                    uint32_t* __restrict__ ent) {
  extern __shared__ __attribute__((aligned(16))) uint32_t fine_lds[];
  const uint32_t wb = MODE == 2 ? gridDim.x - 1 - blockIdx.x : blockIdx.x;
  const uint32_t s0 = bstart[wb], s1 = bstart[wb + 1];
  const bool big = s1 - s0 > kFineCap;  // block-uniform
  if (MODE != 1 && !big) fine_region<true>(tmp, e32, wb, s0, s1, FB, K, gst, tstart, ent, fine_lds);
  if (MODE != 0 && big) fine_region<false>(tmp, e32, wb, s0, s1, FB, K, gst, tstart, ent, fine_lds);
}

// Each thread: K consecutive sorted entries.  See file header.
// Bucket pieces: a bucket whose entries cross thread boundaries is split into an OWNER piece (the
// thread holding its first entry; always that thread's last segment) and HEAD pieces (a later
// thread's first segment).  A bucket of exactly two pieces inside one block -- nearly all of them
// for random scalars -- is joined here: the head goes to LDS, and after the barrier the owner adds
// it to the piece still in its registers (one extra addition per owner at the accumulate's full
// occupancy, no global round trip).  Every other crossing bucket keeps the global pieces
// (pfirst = a thread's first segment, plast = its last) and is queued for k_fixup.  Empty
// buckets are never written: k_wsum reads gst.
static constexpr uint32_t kFixSerial = 8;  // crossing buckets of more pieces: k_fixup's heavy blocks
__device__ __forceinline__ bool join_in_block(uint32_t gs, uint32_t ge, uint32_t K) {
  const uint32_t t0 = gs / K, t1 = (ge - 1) / K;
  return t1 == t0 + 1 && t0 / kBlock == t1 / kBlock;
}
// The accumulator of k_accumulate's chain.  R29 (default): 9 x 29-bit limbs (curve29.hpp; each
// partial product one v_mad_u64_u32 with no carry add, 125 VGPRs = 4 waves per SIMD), reading its
// points from a table already in its form (vtab_put: a limb split per load).  Its bucket sums are STORED in the
// chain's own Montgomery form, x R' as 8 words ("r29w": every coordinate is below 4p < 2^256), not
// converted to field.hpp's canonical x R: a segment end runs for the whole wave whenever one of its
// lanes ends a segment, so its work counts nearly every iteration (the conversion there cost ~70 us
// of a 1.39 ms accumulate).  The readers convert instead: k_fixup (loads and stores r29w, so bsum
// stays uniform for the next host-fed piece), bucket_at (k_wsum, k_wsum_tree<false>, once per
// bucket), and k_wsum_tree<true, true> runs its running sums in the same form (bucket_at29).
// SVGPU_ACC_R29=0 selects the 8 x 32-bit chain (xyzz_madd_2p_u), stored canonical.
#ifndef SV_ACC_MADD32
#define SV_ACC_MADD32 xyzz_madd_2p_u
#endif
template <bool R29>
struct AccChain;
template <>
struct AccChain<false> {
  using T = G1Xyzz;
  __device__ static T identity() { return G1Xyzz::identity(); }
  __device__ static T in(const G1Xyzz& a) { return a; }
  __device__ static G1Xyzz out(const T& a) { return xyzz_canon2p(a); }
  __device__ static T madd(const T& acc, const G1Aff& p, bool neg) {
    return SV_ACC_MADD32(acc, p.x, neg ? -p.y : p.y);
  }
};
template <>
struct AccChain<true> {
  using T = r29::Xyzz;
  __device__ static T identity() { return r29::identity(); }
  __device__ static T in(const G1Xyzz& a) {  // storage form: x R' as words (r29w_*)
    return {r29::from_words(a.X.v), r29::from_words(a.Y.v), r29::from_words(a.ZZ.v), r29::from_words(a.ZZZ.v)};
  }
  __device__ static G1Xyzz out(const T& a) {  // the chain's X may reach 8p: stored below 4p
    G1Xyzz r;
    r29::to_words(r29::csub<4>(a.X), r.X.v);
    r29::to_words(a.Y, r.Y.v);
    r29::to_words(a.ZZ, r.ZZ.v);
    r29::to_words(a.ZZZ, r.ZZZ.v);
    return r;
  }
  __device__ static G1Xyzz canonical(const T& a) {  // field.hpp's canonical x R form
    G1Xyzz r;
    r29::to_r32(r29::csub<4>(a.X), r.X.v);
    r29::to_r32(a.Y, r.Y.v);
    r29::to_r32(a.ZZ, r.ZZ.v);
    r29::to_r32(a.ZZZ, r.ZZZ.v);
    return r;
  }
  __device__ static T madd(const T& acc, const G1Aff& p, bool neg) {
    const r29::F x = r29::from_words(p.x.v), y = r29::from_words(p.y.v);  // the table's x R' words
    return r29::madd(acc, x, y, neg);
  }
};

// SV_ACC_MIN_BLOCKS / SV_ACC29_MIN_BLOCKS: resident 256-thread blocks per CU the register allocator
// must allow for the 8 x 32-bit / 29-bit chains (1: no constraint -- the 32-bit chain takes 144
// VGPRs = 3 waves per SIMD; 4: at most 128 VGPRs, which the 29-bit chain meets without spilling)
#ifndef SV_ACC_MIN_BLOCKS
#define SV_ACC_MIN_BLOCKS 1
#endif
#ifndef SV_ACC29_MIN_BLOCKS
#define SV_ACC29_MIN_BLOCKS 4
#endif
// NL (round 6, the 29-bit chain; the round-5 loop stays for the 32-bit chain only): the chain's state
// is never the identity -- a lane whose chain is empty (segment start, or after P + (-P)) takes its
// next point as the state in the loop's divergent segment-end block and skips that entry's madd, so
// the per-entry step is r29::madd_live with no identity test or identity-valued merge.
template <bool ADD, bool R29, int PF = SV_ACC_PREFETCH, bool NL = R29>  // (R29 implies NL)
__global__ void __launch_bounds__(kBlock, R29 ? SV_ACC29_MIN_BLOCKS : SV_ACC_MIN_BLOCKS) k_accumulate(
    const G1Aff* __restrict__ bases, const uint32_t* __restrict__ ent, const uint32_t* __restrict__ gst,
    const uint32_t* __restrict__ tstart, uint32_t nbt, uint32_t K, uint32_t T,
    G1Xyzz* __restrict__ bsum, G1Xyzz* __restrict__ pfirst, G1Xyzz* __restrict__ plast,
    uint32_t* __restrict__ multi, uint32_t* __restrict__ nmulti, uint32_t* __restrict__ heavy,
    uint32_t* __restrict__ nheavy, const uint4* __restrict__ phix, uint32_t nsplit, int phi64) {
  using A = AccChain<R29>;
  // head pieces for the in-block join: canonical G1Xyzz (32-bit chain) or 29-bit records (144 B)
  __shared__ G1Xyzz shead[R29 ? 1 : kBlock];
  __shared__ uint4 shead29[R29 ? 9 * kBlock : 1];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t m = gst[nbt];
  const uint32_t s0 = t * K;
  const bool active = t < T && s0 < m;
  // owner piece left in acc for the in-block join (g = its bucket), or none
  bool owner = false;
  uint32_t g = 0, gs = 0, ge = 0;
  G1Xyzz sum;  // the last segment's canonical sum (the owner piece's, for the join)
  typename A::T acc = A::identity();
  if (active) {
    const uint32_t e_end = min(s0 + K, m);
    g = tstart[t];
    gs = gst[g];
    ge = gst[g + 1];
    uint32_t seg_start = s0;
    bool first = true;
    // ADD (host-fed pieces after the first): a segment that starts its bucket -- the owner piece --
    // starts from the sum the earlier pieces left in bsum (identity-initialised) instead of the
    // identity, so every later join (in block, k_fixup) and store carries it: no extra addition
    bool empty = true;  // NL: the chain holds no point yet (acc is not read)
    if constexpr (ADD) {
      if (s0 == gs) {
        if constexpr (R29) {
          acc = ld_rec29(bsum, g);
          empty = r29::is_zero(acc.ZZ);
        } else {
          acc = A::in(load_xyzz(bsum, g));
        }
      }
    }
    uint32_t vnext = 0;
    if constexpr (PF >= 1) vnext = ent[s0];
    G1Aff pnext;
    if constexpr (PF >= 2) pnext = load_vpoint(bases, phix, vnext & 0x7fffffffu, nsplit, phi64);
    if constexpr (NL) {
      static_assert(R29 && PF == 1, "the restructured loop is the 29-bit chain's");
      (void)bases;
      (void)nsplit;
      (void)phi64;
      for (uint32_t e = s0; e < e_end; e++) {
        // the entry's point first: a segment starting here starts from it
        const uint32_t v = vnext;
        if (e + 1 < e_end) vnext = ent[e + 1];
        r29::F x, y;  // the table's limbs (the identity: all-zero limbs)
        ld_rec29(reinterpret_cast<const uint2*>(phix) + (size_t)kVtabRec * (v & 0x7fffffffu), x, y);
        const bool live = !(r29::is_zero(x) && r29::is_zero(y)), neg = (v & 0x80000000u) != 0;
        bool fresh = false;
        if (e >= ge || empty) {  // divergent: a segment ends here, or the chain is empty
          if (e >= ge) {  // segment [seg_start, ge) of bucket g ends inside this chunk
            // the state as it is (an empty chain has acc.ZZ == 0, set below / by madd_live's
            // cancellation: the identity)
            if (seg_start == gs) {
              st_rec29(bsum, g, acc);
            } else {  // head piece of a bucket owned by an earlier thread
              if (join_in_block(gs, ge, K)) st_rec29(reinterpret_cast<G1Xyzz*>(shead29), threadIdx.x, acc);
              else st_rec29(pfirst, t, acc);
            }
            first = false;
            do {
              g++;
              gs = ge;
              ge = gst[g + 1];
            } while (ge <= e);
            seg_start = e;
            empty = true;
            if constexpr (ADD) {
              acc = ld_rec29(bsum, g);
              empty = r29::is_zero(acc.ZZ);
            } else {
              acc.ZZ = r29::zero();
            }
          }
          if (empty && live) {
            acc = r29::start(x, y, neg);
            empty = false;
            fresh = true;
          }
        }
        if (live && !fresh) {
          int special = 0;
          acc = r29::madd_live(acc, x, y, neg, special);
          if (special) {  // rare, divergent: P + P, or P + (-P) (the chain restarts at its next point)
            if (special == 2) {
              acc = r29::dbl_start(x, y, neg);
            } else {
              acc.ZZ = r29::zero();  // a chain that ends empty stores the identity
              empty = true;
            }
          }
        }
      }
    } else
    for (uint32_t e = s0; e < e_end; e++) {
      if (e >= ge) {  // segment [seg_start, ge) of bucket g ends inside this chunk
        const G1Xyzz sum = A::out(acc);
        if (seg_start == gs) {
          store_xyzz(bsum, g, sum);
        } else {  // head piece of a bucket owned by an earlier thread
          if (join_in_block(gs, ge, K)) shead[threadIdx.x] = sum;
          else store_xyzz(pfirst, t, sum);
        }
        first = false;
        do {
          g++;
          gs = ge;
          ge = gst[g + 1];
        } while (ge <= e);
        seg_start = e;
        // the new segment starts bucket g (gs == e: entries are contiguous, empty buckets skipped)
        if constexpr (ADD) acc = A::in(load_xyzz(bsum, g));
        else acc = A::identity();
      }
      uint32_t v;
      G1Aff p;
      if constexpr (PF == 0) {
        v = ent[e];
        p = load_vpoint(bases, phix, v & 0x7fffffffu, nsplit, phi64);
      } else if constexpr (PF == 1) {
        v = vnext;
        if (e + 1 < e_end) vnext = ent[e + 1];
        p = load_vpoint(bases, phix, v & 0x7fffffffu, nsplit, phi64);
      } else {
        v = vnext;
        p = pnext;
        if (e + 1 < e_end) {  // next entry's point in flight during this addition
          vnext = ent[e + 1];
          pnext = load_vpoint(bases, phix, vnext & 0x7fffffffu, nsplit, phi64);
        }
      }
      if (!p.is_identity()) acc = A::madd(acc, p, (v & 0x80000000u) != 0);
    }
    if constexpr (!R29) sum = A::out(acc);
    if (seg_start == gs && e_end == ge) {
      if constexpr (R29) st_rec29(bsum, g, acc);
      else store_xyzz(bsum, g, sum);
    } else if (seg_start != gs) {  // first segment, bucket started earlier (it may also go on later)
      if constexpr (R29) {
        if (join_in_block(gs, ge, K)) st_rec29(reinterpret_cast<G1Xyzz*>(shead29), threadIdx.x, acc);
        else st_rec29(pfirst, t, acc);
      } else {
        if (join_in_block(gs, ge, K)) shead[threadIdx.x] = sum;
        else store_xyzz(pfirst, t, sum);
      }
    } else if (join_in_block(gs, ge, K)) {  // this thread owns a two-piece in-block bucket
      owner = true;
    } else {
      if constexpr (R29) st_rec29(first ? pfirst : plast, t, acc);
      else store_xyzz(first ? pfirst : plast, t, sum);
      multi[atomicAdd(nmulti, 1u)] = g;  // joined by k_fixup
      if ((ge - 1) / K - gs / K > kFixSerial) heavy[atomicAdd(nheavy, 1u)] = g;
    }
  }
  __syncthreads();
  if (owner) {
    if constexpr (R29)  // the two pieces added in the chain's own form (r29::add takes X below 12p)
      st_rec29(bsum, g, r29::add(acc, ld_rec29(reinterpret_cast<const G1Xyzz*>(shead29), threadIdx.x + 1)));
    else
      store_xyzz(bsum, g, xyzz_add(sum, shead[threadIdx.x + 1]));
  }
}

// Queued crossing buckets (see k_accumulate): pieces pfirst/plast joined serially when the bucket
// spans at most kFixSerial + 1 threads; longer ones (skewed digits: all-equal scalars, a short top
// window) are queued by k_accumulate for k_fixup's heavy blocks instead of being walked serially.
__device__ __forceinline__ G1Xyzz fixup_head(const G1Xyzz* __restrict__ pfirst, const G1Xyzz* __restrict__ plast,
                                             uint32_t s, uint32_t t0, uint32_t K, int r29w) {
  return load_bucket((s == t0 * K) ? pfirst : plast, t0, r29w);
}

// One launch for both queues: blocks [0, gm) walk the multi queue (grid-stride, one bucket per
// thread, a serial chain of at most kFixSerial 2p-domain additions), blocks [gm, gridDim) take the
// heavy queue (one bucket per block: strided partial sums of the per-thread pieces + LDS tree).
// The two queues hold disjoint buckets (k_accumulate puts a bucket of more than kFixSerial + 1
// pieces in both; the multi walk skips it).
__global__ void __launch_bounds__(kBlock) k_fixup(const uint32_t* __restrict__ gst, uint32_t K,
                                                  const G1Xyzz* __restrict__ pfirst,
                                                  const G1Xyzz* __restrict__ plast,
                                                  const uint32_t* __restrict__ multi,
                                                  const uint32_t* __restrict__ nmulti,
                                                  const uint32_t* __restrict__ heavy,
                                                  const uint32_t* __restrict__ nheavy, uint32_t gm,
                                                  G1Xyzz* __restrict__ bsum, int r29w) {
  __shared__ G1Xyzz sh[kBlock];
  const uint32_t tid = threadIdx.x;
  if (blockIdx.x < gm) {  // block-uniform
    // one bucket per QUAD of lanes (quad.hpp: lane c = coordinate c): the chain of at most
    // kFixSerial additions is latency-bound (a few waves per SIMD), so 4-level quad additions
    // shorten it 2-3x; every branch below is uniform within the quad
    const uint32_t nm = *nmulti;
    const int c = tid & 3;
    for (uint32_t h = (blockIdx.x * blockDim.x + tid) >> 2; h < nm; h += (gm * blockDim.x) >> 2) {
      const uint32_t g = multi[h];
      const uint32_t s = gst[g], e = gst[g + 1];
      const uint32_t t0 = s / K, t1 = (e - 1) / K;
      if (t1 - t0 > kFixSerial) continue;  // a heavy bucket: the other blocks' part
      // r29w (k_accumulate's 29-bit chain): pieces and the stored sum as 29-bit records
      const G1Xyzz* h0 = s == t0 * K ? pfirst : plast;
      Fq acc = r29w ? rec29_coord_canonical(rec_at(h0, t0, 1), c) : quad::ld(h0 + t0, c);
      for (uint32_t t = t0 + 1; t <= t1; t++) {
        const Fq v = r29w ? rec29_coord_canonical(rec_at(pfirst, t, 1), c) : quad::ld(pfirst + t, c);
        acc = quad::add_2p(acc, v, c);
      }
      acc = fe_canon2p(acc);
      if (r29w) rec29_coord_store(rec_at(bsum, g, 1), c, acc);
      else quad::st(bsum + g, c, acc);
    }
    return;
  }
  const uint32_t nh = *nheavy, gh = gridDim.x - gm;
  for (uint32_t h = blockIdx.x - gm; h < nh; h += gh) {
    const uint32_t g = heavy[h];
    const uint32_t s = gst[g], e = gst[g + 1];
    const uint32_t t0 = s / K, t1 = (e - 1) / K;
    G1Xyzz acc = G1Xyzz::identity();
    for (uint32_t t = t0 + 1 + tid; t <= t1; t += kBlock) acc = xyzz_add(acc, load_bucket(pfirst, t, r29w));
    sh[tid] = acc;
    __syncthreads();
    for (uint32_t st = kBlock / 2; st > 0; st >>= 1) {
      if (tid < st) sh[tid] = xyzz_add(sh[tid], sh[tid + st]);
      __syncthreads();
    }
    if (tid == 0) {
      const G1Xyzz sum = xyzz_add(fixup_head(pfirst, plast, s, t0, K, r29w), sh[0]);
      store_bucket(bsum, g, xyzz_canon2p(sum), r29w);
    }
    __syncthreads();
  }
}

// Bucket i of one window (x, gs: that window's bucket sums and starts): false when empty.
// gs == null: every bucket was written (host-fed merge).  (Joining the crossing buckets here
// instead of in k_fixup was measured 155 -> 440 us for k_wsum at 2^20: ~7 % of buckets cross,
// so nearly every wave's iteration diverges into the join loop.)
__device__ __forceinline__ bool bucket_at(const G1Xyzz* __restrict__ x, const uint32_t* __restrict__ gs, uint32_t i,
                                          G1Xyzz& out, int r29w) {  // r29w: sums in the 29-bit chain's form
  if (gs && gs[i] == gs[i + 1]) return false;
  out = load_bucket(x, i, r29w);
  return true;
}

// bucket i in the 29-bit chain's own form (its record as stored: no conversion); false when empty
__device__ __forceinline__ bool bucket_at29(const G1Xyzz* __restrict__ x, const uint32_t* __restrict__ gs, uint32_t i,
                                            r29::Xyzz& out) {
  if (gs && gs[i] == gs[i + 1]) return false;
  out = ld_rec29(x, i);
  return true;
}

// One bucket-reduction level over `groups` groups of N elements, segments of L buckets:
//   acc[g][j] = sum_{i in seg j} (i - jL + base) X[g][i],  tot[g][j] = sum_{i in seg j} X[g][i]
// Empty buckets (gst[b] == gst[b + 1]) are never written by the accumulate pass and read as identity.
__global__ void __launch_bounds__(kBlock) k_wsum(const G1Xyzz* __restrict__ X, const uint32_t* __restrict__ gst,
                                                 uint32_t N, uint32_t J, uint32_t L, uint32_t groups, int base,
                                                 G1Xyzz* __restrict__ acc_out, G1Xyzz* __restrict__ tot_out,
                                                 int r29w) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= J * groups) return;
  uint32_t g = tid / J, j = tid % J;
  const G1Xyzz* x = rec_at(X, (size_t)g * N, r29w);
  const uint32_t* gs = gst ? gst + (size_t)g * N : nullptr;
  uint32_t lo = j * L;
  uint32_t hi = min(N, lo + L);
  G1Xyzz run = G1Xyzz::identity(), acc = G1Xyzz::identity();
  if (hi > lo) {
    // bucket i - 1 (and its emptiness) is loaded while bucket i is being added (A/B at 2^20:
    // reduce 0.404 -> 0.393 ms)
    uint32_t i = hi - 1;
    G1Xyzz nx = G1Xyzz::identity();
    bool ne = bucket_at(x, gs, i, nx, r29w);
    for (;;) {
      const G1Xyzz cur = nx;
      const bool cne = ne;
      const uint32_t ci = i;
      if (ci > lo) {
        i = ci - 1;
        ne = bucket_at(x, gs, i, nx, r29w);
      }
      if (cne) run = xyzz_add_2p(run, cur);
      if (base || ci > lo) acc = xyzz_add_2p(acc, run);
      if (ci == lo) break;
    }
  }
  store_xyzz(acc_out, tid, xyzz_canon2p(acc));
  if (tot_out) store_xyzz(tot_out, tid, xyzz_canon2p(run));
}

// Step 2 fused: P 512-thread blocks per (window, group) each sum a 1/P slice of the group's H
// members (strided, ~H/(512 P) serial adds per thread) and finish with an LDS tree (9 levels).
// With P > 1 the slices' sums go to part[] and the block that finishes last (device-scope counter
// cnt[gid], zeroed per call) adds them -> out[w*NG + q].  P = 2 whenever the groups alone would not
// give every CU a block (GLV at 2^20: 120 groups, 17 -> 13 dependent additions per chain).
static constexpr int kGroupBlock = 512;
// member m of group q of window w (see above)
__device__ __forceinline__ G1Xyzz group_member(const G1Xyzz* __restrict__ acc, const G1Xyzz* __restrict__ tot,
                                               uint32_t w, uint32_t q, uint32_t J, uint32_t H, uint32_t m) {
  if (q < 2) return load_xyzz(acc, w * J + q * H + m);
  const uint32_t k = q - 2;
  const uint32_t j = ((m >> k) << (k + 1)) | (1u << k) | (m & ((1u << k) - 1));
  return load_xyzz(tot, w * J + j);
}
// XYZZ value of one lane as 32 dwords: LDS in structure-of-arrays order (dword d of lane t at
// [d][t], conflict-free), and a wave-level shift down by `off` lanes
__device__ __forceinline__ void sh_put(uint32_t (*sh)[kGroupBlock], uint32_t t, const G1Xyzz& v) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < 32; k++) sh[k][t] = d[k];
}
__device__ __forceinline__ G1Xyzz sh_get(uint32_t (*sh)[kGroupBlock], uint32_t t) {
  G1Xyzz v;
  uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < 32; k++) d[k] = sh[k][t];
  return v;
}
__device__ __forceinline__ G1Xyzz wave_down(const G1Xyzz& v, int off) {
  G1Xyzz r;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int k = 0; k < 32; k++) o[k] = __shfl_down(d[k], off);
  return r;
}
__global__ void __launch_bounds__(kGroupBlock) k_group_sum(const G1Xyzz* __restrict__ acc,
                                                           const G1Xyzz* __restrict__ tot, uint32_t J,
                                                           uint32_t logJ, uint32_t P, G1Xyzz* __restrict__ out,
                                                           G1Xyzz* __restrict__ part, uint32_t* __restrict__ cnt) {
  __shared__ uint32_t sh[32][kGroupBlock];  // 64 KiB
  const uint32_t NG = 2 + logJ, H = J / 2;
  const uint32_t gid = blockIdx.x / P, pp = blockIdx.x % P, w = gid / NG, q = gid % NG, tid = threadIdx.x;
  const uint32_t m0 = (uint32_t)((uint64_t)H * pp / P), m1 = (uint32_t)((uint64_t)H * (pp + 1) / P);
  // strided members, two loads in flight per addition pair
  G1Xyzz s = G1Xyzz::identity();
  uint32_t m = m0 + tid;
  for (; m + kGroupBlock < m1; m += 2 * kGroupBlock) {
    const G1Xyzz x0 = group_member(acc, tot, w, q, J, H, m);
    const G1Xyzz x1 = group_member(acc, tot, w, q, J, H, m + kGroupBlock);
    s = xyzz_add_2p(s, x0);
    s = xyzz_add_2p(s, x1);
  }
  if (m < m1) s = xyzz_add_2p(s, group_member(acc, tot, w, q, J, H, m));
  // tree: three cross-wave levels through LDS, then six inside wave 0
  for (uint32_t st = kGroupBlock / 2; st >= 64; st >>= 1) {
    if (tid >= st && tid < 2 * st) sh_put(sh, tid, s);
    __syncthreads();
    if (tid < st) s = xyzz_add_2p(s, sh_get(sh, tid + st));
    __syncthreads();
  }
  if (tid >= 64) return;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const G1Xyzz o = wave_down(s, off);
    if ((int)tid < off) s = xyzz_add_2p(s, o);
  }
  if (tid != 0) return;
  if (P > 1) {
    store_xyzz(part, blockIdx.x, s);
    __threadfence();
    if (atomicAdd(&cnt[gid], 1u) != P - 1) return;
    __threadfence();
    for (uint32_t k = 0; k < P; k++)
      if (k != pp) s = xyzz_add_2p(s, load_xyzz(part, gid * P + k));
  }
  store_xyzz(out, gid, xyzz_canon2p(s));
}

// The same subset sums with every XYZZ addition split over a quad of lanes (quad.hpp: lane
// c = lane & 3 holds coordinate c; 4 product levels per addition instead of ~14 dependent products):
// the tree is latency-bound (one wave per SIMD, most lanes idle in its upper levels), so a 3-4x
// shorter addition shortens the whole kernel.  512-thread blocks: strided member sums with whole
// per-lane additions (4 per lane: throughput work), then the tree in quad form -- a 4 x 4 transpose
// turns each quad's four sums into quad-form points (two levels), then four in-wave levels (lane
// shifts of 32 .. 4) and three cross-wave levels through LDS: 9 quad-addition levels instead of 9
// whole-addition levels.
__global__ void __launch_bounds__(kGroupBlock) k_group_sum_q(const G1Xyzz* __restrict__ acc,
                                                             const G1Xyzz* __restrict__ tot, uint32_t J,
                                                             uint32_t logJ, uint32_t P, G1Xyzz* __restrict__ out,
                                                             G1Xyzz* __restrict__ part, uint32_t* __restrict__ cnt) {
  constexpr int kWaves = kGroupBlock / 64;
  __shared__ Fq sh[kWaves][4];
  const uint32_t NG = 2 + logJ, H = J / 2;
  const uint32_t gid = blockIdx.x / P, pp = blockIdx.x % P, w = gid / NG, g = gid % NG, tid = threadIdx.x;
  const int c = tid & 3, lane = tid & 63, wave = tid >> 6;
  const uint32_t m0 = (uint32_t)((uint64_t)H * pp / P), m1 = (uint32_t)((uint64_t)H * (pp + 1) / P);
  // strided member sums with whole additions per lane (throughput work: every lane busy), two loads
  // in flight per addition pair, as k_group_sum
  G1Xyzz ps = G1Xyzz::identity();
  uint32_t m = m0 + tid;
  for (; m + kGroupBlock < m1; m += 2 * kGroupBlock) {
    const G1Xyzz x0 = group_member(acc, tot, w, g, J, H, m);
    const G1Xyzz x1 = group_member(acc, tot, w, g, J, H, m + kGroupBlock);
    ps = xyzz_add_2p(ps, x0);
    ps = xyzz_add_2p(ps, x1);
  }
  if (m < m1) ps = xyzz_add_2p(ps, group_member(acc, tot, w, g, J, H, m));
  // the tree in quad form: transpose the quad's four points to coordinates, add them (two levels),
  // then quads across the wave and across waves
  Fq v[4] = {ps.X, ps.Y, ps.ZZ, ps.ZZZ};
  quad::transpose(v, c);
  Fq s = quad::add_2p(quad::add_2p(v[0], v[1], c), quad::add_2p(v[2], v[3], c), c);
#pragma unroll 1
  for (int off = 32; off >= 4; off >>= 1) {
    const Fq o = quad::down(s, off);
    if (lane < off) s = quad::add_2p(s, o, c);
  }
  if (lane < 4) sh[wave][c] = s;
  __syncthreads();
  if (wave != 0) return;
  if (lane < 4 * kWaves) s = sh[lane >> 2][c];
#pragma unroll 1
  for (int off = 2 * kWaves; off >= 4; off >>= 1) {
    const Fq o = quad::down(s, off);
    if (lane < off) s = quad::add_2p(s, o, c);
  }
  if (lane >= 4) return;
  if (P > 1) {
    quad::st(part + blockIdx.x, c, s);
    __threadfence();
    uint32_t prev = 0;
    if (lane == 0) prev = atomicAdd(&cnt[gid], 1u);
    prev = (uint32_t)__shfl((int)prev, 0);
    if (prev != P - 1) return;  // uniform over the quad
    __threadfence();
    for (uint32_t k = 0; k < P; k++)
      if (k != pp) s = quad::add_2p(s, quad::ld(part + gid * P + k, c), c);
  }
  quad::st(out + gid, c, fe_canon2p(s));
}

// ---- Round 3: the subset sums as a tree inside the running-sum kernel.  k_group_sum(_q) sums every
// group U_k = sum_{j : bit k of j} T_j from scratch: logJ groups of J/2 members, ~J logJ / 2 additions
// per window.  The tree shares them: with block sums BS_0 = T, BS_{l+1}[i] = BS_l[2i] + BS_l[2i+1],
// U_l = sum of the odd BS_l[i] -- ~2J additions per window (and A = sum_j acc_j).  k_wsum_tree runs
// the running sums of 256 consecutive segments per block (one per thread, as k_wsum) and then the
// tree of the block's 256 segments in LDS, in place: at level l the pair (2i, 2i+1) of 2^l-blocks
// merges BS into position 2i 2^l, leaves its right half's sum at (2i + 1) 2^l as U_l's partial, and
// merges the partials of every U_k, k < l, at offset 2^k of the two halves -- (2 + l) 2^(7-l) tasks
// (A, BS, U_0..U_(l-1)), reads only from right halves, writes only to left halves, so a level needs
// one barrier.  Level 0 runs in registers (lane pairs, whole additions); levels 1..7 in quad form.
// A block ends with 10 points: A, the block total CT and U_0..U_7's partials (positions 2^k).
// k_group_fin then sums them per window: A over the blocks (two halves, the A_lo / A_hi slots the
// host Horner expects), U_k (k < 8) over the blocks, U_k (k >= 8) over the blocks whose index has
// bit k - 8 set (their CT).
static constexpr int kTreeLog = 8, kTreeN = 1 << kTreeLog;  // segments per block (= threads)
static constexpr int kTreeRS = kTreeN + 1;                  // LDS row stride in dwords (quads conflict-free)
static constexpr int kTreeOut = 2 + kTreeLog;               // per-block outputs
static constexpr size_t kTreeRow = (size_t)32 * kTreeRS * 4;  // one row of 256 points, structure of arrays

// dword d of point p at row[d * kTreeRS + p]; the quad form reads coordinate c (dwords 8c .. 8c + 7)
__device__ __forceinline__ void tr_put(uint32_t* row, uint32_t p, const G1Xyzz& v) {
  const uint32_t* d = reinterpret_cast<const uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < 32; k++) row[k * kTreeRS + p] = d[k];
}
__device__ __forceinline__ G1Xyzz tr_get(const uint32_t* row, uint32_t p) {
  G1Xyzz v;
  uint32_t* d = reinterpret_cast<uint32_t*>(&v);
#pragma unroll
  for (int k = 0; k < 32; k++) d[k] = row[k * kTreeRS + p];
  return v;
}
__device__ __forceinline__ Fq tr_getc(const uint32_t* row, uint32_t p, int c) {
  Fq r;
#pragma unroll
  for (int k = 0; k < 8; k++) r.v[k] = row[(8 * c + k) * kTreeRS + p];
  return r;
}
__device__ __forceinline__ void tr_putc(uint32_t* row, uint32_t p, int c, const Fq& v) {
#pragma unroll
  for (int k = 0; k < 8; k++) row[(8 * c + k) * kTreeRS + p] = v.v[k];
}
__device__ __forceinline__ G1Xyzz xor1(const G1Xyzz& v) {  // the neighbour lane's point (DPP quad_perm)
  G1Xyzz r;
  const uint32_t* d = reinterpret_cast<const uint32_t*>(&v);
  uint32_t* o = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
  for (int k = 0; k < 32; k++) o[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)d[k], quad::qp(1, 0, 3, 2), 0xF, 0xF, false);
  return r;
}
// task tau of tree level l (pairs of 2^l-blocks, np pairs, A row first when RUN): its row and the
// left-half slot it merges into (the right half's slot is + 2^l)
template <bool RUN>
__device__ __forceinline__ uint32_t* tr_task(uint32_t tau, uint32_t np, uint32_t s, uint32_t* rowA, uint32_t* rowT,
                                             uint32_t& dst) {
  if (RUN && tau < np) {
    dst = 2 * tau * s;
    return rowA;
  }
  const uint32_t r = RUN ? tau - np : tau, kk = r / np, i = r % np;  // kk 0: BS, kk >= 1: U_(kk-1) at 2^(kk-1)
  dst = 2 * i * s + (kk ? 1u << (kk - 1) : 0u);
  return rowT;
}

// RUN: running sums over L-bucket segments, then the tree over the block's 256 segments (rows A and
// T; one block per CU at 2^20).  !RUN (round 3, L = 1): the tree straight over 256 buckets per block
// -- no running sums and no A row (A = the total), a quarter of the LDS, so four blocks share a CU
// and one block's latency-bound upper levels overlap another's wide lower ones; its wide levels
// 1 and 2 run as whole additions (one per lane), the rest in quad form.
template <bool RUN, bool R29 = false>
__global__ void __launch_bounds__(kTreeN) k_wsum_tree(const G1Xyzz* __restrict__ X, const uint32_t* __restrict__ gst,
                                                       uint32_t N, uint32_t J, uint32_t L,
                                                       G1Xyzz* __restrict__ blk_out, int r29w) {
  extern __shared__ uint32_t tr_lds[];
  uint32_t* rowT = tr_lds;
  uint32_t* rowA = tr_lds + 32 * kTreeRS;  // RUN only
  constexpr int kWhole = RUN ? 1 : 3;      // levels below this run as whole additions
  const uint32_t tid = threadIdx.x, bpw = J >> kTreeLog;
  const uint32_t g = blockIdx.x / bpw, j = (blockIdx.x % bpw) * kTreeN + tid;
  const G1Xyzz* x = rec_at(X, (size_t)g * N, r29w);
  const uint32_t* gs = gst ? gst + (size_t)g * N : nullptr;
  const bool odd = tid & 1;
  if constexpr (RUN) {
    // running sums over segment j of window g, exactly as k_wsum with base 1
    const uint32_t lo = j * L, hi = min(N, lo + L);
    G1Xyzz run = G1Xyzz::identity(), acc = G1Xyzz::identity();
    if constexpr (R29) {
      // the 29-bit chain's sums (r29w) read as they are stored, the running sums in the same form
      // (r29::add: no carry adds, no per-bucket conversion), converted once for the tree below
      r29::Xyzz run29 = r29::identity(), acc29 = r29::identity();
      if (hi > lo) {
        uint32_t i = hi - 1;
        r29::Xyzz nx = r29::identity();
        bool ne = bucket_at29(x, gs, i, nx);
        for (;;) {
          const r29::Xyzz cur = nx;
          const bool cne = ne;
          const uint32_t ci = i;
          if (ci > lo) {
            i = ci - 1;
            ne = bucket_at29(x, gs, i, nx);
          }
          if (cne) run29 = r29::add(run29, cur);
          acc29 = r29::add(acc29, run29);
          if (ci == lo) break;
        }
      }
      run = AccChain<true>::canonical(run29);
      acc = AccChain<true>::canonical(acc29);
    } else if (hi > lo) {
      uint32_t i = hi - 1;
      G1Xyzz nx = G1Xyzz::identity();
      bool ne = bucket_at(x, gs, i, nx, r29w);
      for (;;) {
        const G1Xyzz cur = nx;
        const bool cne = ne;
        const uint32_t ci = i;
        if (ci > lo) {
          i = ci - 1;
          ne = bucket_at(x, gs, i, nx, r29w);
        }
        if (cne) run = xyzz_add_2p(run, cur);
        acc = xyzz_add_2p(acc, run);
        if (ci == lo) break;
      }
    }
    // level 0 (lane pairs, one addition per lane): even lanes A[2i] + A[2i+1], odd lanes
    // T[2i] + T[2i+1]; the odd T stays where it is as U_0's partial
    const G1Xyzz oa = xor1(acc), ot = xor1(run);
    const G1Xyzz s0 = xyzz_add_2p(odd ? ot : acc, odd ? run : oa);
    if (odd) {
      tr_put(rowT, tid - 1, s0);
      tr_put(rowT, tid, run);
    } else {
      tr_put(rowA, tid, s0);
    }
  } else {
    // level 0 over the buckets themselves (odd lanes; an empty bucket is the identity)
    G1Xyzz t = G1Xyzz::identity();
    if (j < N) bucket_at(x, gs, j, t, r29w);
    const G1Xyzz ot = xor1(t);
    if (odd) {
      tr_put(rowT, tid - 1, xyzz_add_2p(ot, t));
      tr_put(rowT, tid, t);
    }
  }
  __syncthreads();
  const int c = tid & 3;
  const uint32_t qd = tid >> 2;
#pragma unroll 1
  for (int l = 1; l < kTreeLog; l++) {
    const uint32_t s = 1u << l, np = (uint32_t)kTreeN >> (l + 1), ntask = ((RUN ? 2 : 1) + l) * np;
    if (l < kWhole) {  // whole additions, one task per thread (ntask <= 256)
      if (tid < ntask) {
        uint32_t dst;
        uint32_t* row = tr_task<RUN>(tid, np, s, rowA, rowT, dst);
        const G1Xyzz a = tr_get(row, dst), b = tr_get(row, dst + s);
        tr_put(row, dst, xyzz_add_2p(a, b));
      }
    } else {  // quad form: a task per quad and round (tasks of one level touch disjoint slots)
#pragma unroll 1
      for (uint32_t tau = qd; tau < ntask; tau += kTreeN / 4) {
        uint32_t dst;
        uint32_t* row = tr_task<RUN>(tau, np, s, rowA, rowT, dst);
        const Fq a = tr_getc(row, dst, c), b = tr_getc(row, dst + s, c);
        tr_putc(row, dst, c, quad::add_2p(a, b, c));
      }
    }
    __syncthreads();
  }
  // [A,] CT, U_0 .. U_7 -> blk_out (2p domain; k_group_fin canonicalises)
  if (tid >= (RUN ? 0u : 4u) && tid < (uint32_t)kTreeOut * 4) {
    const uint32_t q = tid >> 2;
    const uint32_t* row = q == 0 ? rowA : rowT;
    const uint32_t p = q < 2 ? 0u : 1u << (q - 2);
    quad::st(blk_out + (size_t)blockIdx.x * kTreeOut + q, c, tr_getc(row, p, c));
  }
}

// One block of two waves per (window, output slot): up to 128 members (bpw = J / 256 <= 128), each
// wave's 64 transposed into quad form, two quad additions inside each quad, the in-wave levels that
// still hold members, then wave 1's sum added to wave 0's.  aslot: the per-block slot the A sums
// read (0: A with running sums, 1: the block total CT for the pure tree).
__global__ void __launch_bounds__(128) k_group_fin(const G1Xyzz* __restrict__ blk_out, uint32_t bpw, uint32_t NG,
                                                   uint32_t aslot, G1Xyzz* __restrict__ out) {
  __shared__ Fq sh[4];
  const uint32_t w = blockIdx.x / NG, q = blockIdx.x % NG, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = lane & 3;
  const G1Xyzz* bo = blk_out + (size_t)w * bpw * kTreeOut;
  uint32_t members, b = tid, slot;
  if (q < 2) {  // A over the first / second half of the window's blocks
    const uint32_t h = (bpw + 1) / 2;
    members = q == 0 ? h : bpw - h;
    b = (q == 0 ? 0 : h) + tid;
    slot = aslot;
  } else if (q - 2 < (uint32_t)kTreeLog) {  // U_k, k < 8: every block's partial
    members = bpw;
    slot = q;
  } else {  // U_k, k >= 8: the totals of the blocks with bit k - 8 set
    const uint32_t m = q - 2 - kTreeLog;
    members = bpw / 2;
    b = ((tid >> m) << (m + 1)) | (1u << m) | (tid & ((1u << m) - 1));
    slot = 1;
  }
  if (wv > 0 && wv * 64 >= members) return;  // wave 1 only when there are more than 64 (wave 0 always
                                              // stores, the identity for an empty slot)
  const G1Xyzz v = tid < members ? load_xyzz(bo, b * kTreeOut + slot) : G1Xyzz::identity();
  Fq t[4] = {v.X, v.Y, v.ZZ, v.ZZZ};
  quad::transpose(t, c);
  Fq s = quad::add_2p(quad::add_2p(t[0], t[1], c), quad::add_2p(t[2], t[3], c), c);
  const uint32_t wm = min(64u, members - wv * 64);
  const uint32_t live = (wm + 3) / 4 * 4;  // lanes whose quads hold members
#pragma unroll 1
  for (uint32_t off = 32; off >= 4; off >>= 1) {
    if (off >= live) continue;  // uniform: only identities above
    const Fq o = quad::down(s, off);
    if (lane < off) s = quad::add_2p(s, o, c);
  }
  if (members > 64) {
    if (wv == 1 && lane < 4) sh[c] = s;
    __syncthreads();
    if (wv == 1) return;
    const Fq o = sh[c];
    s = quad::add_2p(s, o, c);
  }
  if (lane < 4) quad::st(out + blockIdx.x, c, fe_canon2p(s));
}

// ---------------------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------------------
static thread_local sv_msm_stats g_last_stats;

int msm_last_stats(sv_msm_stats* out) {
  *out = g_last_stats;
  return SV_OK;
}

static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

// Sorted entries per accumulate thread for `entries` entries over nbt buckets (SVGPU_ACC_K forces it)
static uint32_t plan_K(uint64_t entries, uint32_t nbt) {
  uint64_t K = entries / (1u << 18);
  if (K < 4) K = 4;
  if (K > 32) K = 32;
  // large n: buckets average entries / nbt > 32 entries; a chunk of about one average bucket keeps
  // most crossing buckets at two pieces (joined inside k_accumulate), capped at 256 entries so the
  // grid still has many rounds of waves (swept, tools/gpu_sweep_big.sh: 2^21 K = 64 4.47 -> 4.41 ms;
  // 2^24 K = 256 32.0 ms, 512 32.4, 1024 33.4)
  const uint64_t avg_bucket = entries / nbt;
  if (K < avg_bucket) K = avg_bucket < 256 ? avg_bucket : 256;
  if (const char* e = getenv("SVGPU_ACC_K")) K = (uint64_t)atoi(e);
  if (K < 1) K = 1;
  return (uint32_t)K;
}

// Host-fed pieces (a fraction of the points over the whole bucket set, so few entries per bucket):
// chunks of about one average bucket, a multiple of 8, at least 16.  Round 3 (the 32-bit chain,
// measured device-resident at the 2^20 plan's window) had found about two average buckets best while
// that stayed <= 32 entries: a segment end then cost ~110 VALU instructions.  With the round-6
// chain's raw-record segment ends, a quarter-size piece's accumulate at K = 32 filled only half the
// chip's block slots; one average bucket (K = 24, 16, 16, 16 for the 2^20 pieces 5,4,4,3) measured
// 2.538-2.570 ms per host-fed 2^20 MSM against 2.602-2.609 (SVGPU_ACC_K = 16 for every piece, two
// passes, profiles/r06_host_piece_k.log).
static uint32_t piece_K(uint64_t entries, uint32_t nbt) {
  if (getenv("SVGPU_ACC_K")) return plan_K(entries, nbt);
  const uint64_t avg = entries / nbt;
  const uint64_t K = std::min<uint64_t>(std::max<uint64_t>((avg + 7) / 8 * 8, 16), 256);
  return (uint32_t)K;
}

MsmPlan msm_plan(size_t n) {
  MsmPlan p;
  // GLV (k P = k1 P + k2 phi(P), 128-bit halves, split on the fly by the sort passes) halves the
  // buckets, the bucket reduction and the host Horner for the same number of bucket entries, at the
  // cost of a 32-B beta-x table per point.  Measured (r02, med ms, GLV off -> on): 2^14 0.79 -> 0.74,
  // 2^16 0.98 -> 0.82, 2^18 1.75 -> 1.54, 2^20 2.11 -> 2.05, 2^21 3.74 -> 3.62; at 2^22 (6.88 ->
  // 7.39) and 2^24 (27.3 -> 31.1) the larger gather working set (bases + beta-x beyond the 256 MiB
  // Infinity Cache) slows the fill, so it is on up to 2^SVGPU_GLV_MAX_LOG points (default 21);
  // SVGPU_GLV forces it.
  int glv_max_log = 21;
  if (const char* e = getenv("SVGPU_GLV_MAX_LOG")) glv_max_log = atoi(e);
  p.glv = n >= (size_t(1) << 14) && n <= (size_t(1) << glv_max_log);
  if (const char* e = getenv("SVGPU_GLV")) p.glv = atoi(e) != 0 && n >= 2;
  p.npts = p.glv ? 2 * n : n;
  // whole phi(P) records (one 64-B gather per k2 entry) while bases + table stay well inside the
  // Infinity Cache; beta-x only above (measured at 2^20: 1.97-2.01 vs 2.01-2.15 ms, k_accumulate
  // 1.39 vs 1.39-1.50 ms)
  p.phi64 = n <= (size_t(1) << 20);
  if (const char* e = getenv("SVGPU_GLV_PHI64")) p.phi64 = atoi(e) != 0;
  const int nb = p.glv ? 128 : 255;
  int lg = 0;
  while ((size_t(1) << (lg + 1)) <= p.npts) lg++;
  int c = lg - 4;
  if (const char* e = getenv("SVGPU_WINDOW_BITS")) c = atoi(e);
  if (c < 4) c = 4;
  if (c > 16) c = 16;
  p.c = c;
  p.W = (nb + c - 1) / c;
  p.B = 1u << (c - 1);
  p.nbt = p.B * p.W;
  uint64_t entries = (uint64_t)p.npts * p.W;
  p.K = plan_K(entries, p.nbt);
  p.T = cdiv(entries, p.K);
  // reduction: J running-sum segments per window, NG subset groups of H = J/2 points
  // 8 buckets per running-sum segment (swept: tools/gpu_sweep_red.sh); 4 with GLV, whose W / 2
  // windows would otherwise leave half the SIMDs without a k_wsum wave
  p.logL = p.glv ? 2 : 3;
  if (const char* e = getenv("SVGPU_RED_LOG")) p.logL = atoi(e);
  if (p.logL < 1) p.logL = 1;
  if (p.logL > p.c - 3) p.logL = p.c - 3 > 1 ? p.c - 3 : 1;
  // bucket reduction (SVGPU_GROUP_TREE): 1 (default) running sums + in-block subset-sum tree
  // (k_wsum_tree<true>) when a window's segments fill whole 256-segment blocks, at most 64 of them;
  // 2 the tree straight over the buckets (k_wsum_tree<false>, no running sums: L = 1); 0 k_wsum +
  // k_group_sum(_q)
  p.tree = 1;
  if (const char* e = getenv("SVGPU_GROUP_TREE")) p.tree = atoi(e);
  // k_accumulate's chain (AccChain): the 29-bit one unless SVGPU_ACC_R29=0; fixed per call, so
  // the accumulate, fixup and reduction launches of one MSM agree on the stored form
  p.r29 = !getenv("SVGPU_ACC_R29") || atoi(getenv("SVGPU_ACC_R29")) != 0;
  if (p.tree == 2 && p.B % kTreeN == 0 && p.B / kTreeN <= 128) p.logL = 0;
  else if (p.tree == 2) p.tree = 1;
  p.J = p.B >> p.logL;
  if (p.tree == 1 && !(p.J % kTreeN == 0 && p.J / kTreeN <= 64)) p.tree = 0;
  p.logJ = 0;
  while ((1u << p.logJ) < p.J) p.logJ++;
  p.NG = 2 + p.logJ;
  return p;
}

#define SV_LAUNCH_LOGB(KERNEL, LOGB, GRID, BLOCK, ...)                          \
  switch (LOGB) {                                                              \
    case 3: hipLaunchKernelGGL(KERNEL<3>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 4: hipLaunchKernelGGL(KERNEL<4>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 5: hipLaunchKernelGGL(KERNEL<5>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 6: hipLaunchKernelGGL(KERNEL<6>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 7: hipLaunchKernelGGL(KERNEL<7>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 8: hipLaunchKernelGGL(KERNEL<8>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 9: hipLaunchKernelGGL(KERNEL<9>, GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 10: hipLaunchKernelGGL(KERNEL<10>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 11: hipLaunchKernelGGL(KERNEL<11>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 12: hipLaunchKernelGGL(KERNEL<12>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 13: hipLaunchKernelGGL(KERNEL<13>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 14: hipLaunchKernelGGL(KERNEL<14>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 15: hipLaunchKernelGGL(KERNEL<15>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    default: break;                                                            \
  }

#define SV_LAUNCH_C1(KERNEL, G, C, GRID, BLOCK, ...)                                              \
  switch (C) {                                                                                   \
    case 4: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<4, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 5: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<5, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 6: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<6, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 7: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<7, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 8: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<8, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 9: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<9, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break;   \
    case 10: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<10, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 11: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<11, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 12: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<12, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 13: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<13, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 14: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<14, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 15: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<15, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    case 16: hipLaunchKernelGGL(HIP_KERNEL_NAME(KERNEL<16, G>), GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    default: break;                                                                              \
  }
// full scalars or GLV halves (split on the fly)
#define SV_LAUNCH_C(KERNEL, GLV, C, GRID, BLOCK, ...)              \
  if (GLV) {                                                       \
    SV_LAUNCH_C1(KERNEL, true, C, GRID, BLOCK, __VA_ARGS__)        \
  } else {                                                         \
    SV_LAUNCH_C1(KERNEL, false, C, GRID, BLOCK, __VA_ARGS__)       \
  }

// Host Horner over every exponent: the group sums of window w are A_lo, A_hi at 2^(c w) and U_k at
// 2^(c w + logL + k), k < logJ (logL + logJ = c - 1, so the windows' exponents never collide), so one
// chain of c (W - 1) + c - 2 doublings with each term added at its exponent computes the total --
// 126 doublings + 120 additions with GLV at 2^20 instead of 224 + 119 for a Horner per window
// followed by one over the windows.
static host::Xyzz host_combine(const MsmPlan& p, const host::Xyzz* A) {
  const int top = (int)((p.W - 1) * p.c + p.logL + p.logJ - 1);
  host::Xyzz acc = host::x_identity();
  for (int e = top; e >= 0; e--) {
    acc = host::x_dbl(acc);
    const uint32_t w = (uint32_t)e / p.c, r = (uint32_t)e % p.c;
    const host::Xyzz* a = A + w * p.NG;
    if (r == 0) acc = host::x_add(host::x_add(acc, a[0]), a[1]);
    // (the tree straight over the buckets has logL = 0: U_0 shares A's exponent)
    if (r >= p.logL && r - p.logL < p.logJ) acc = host::x_add(acc, a[2 + r - p.logL]);
  }
  return acc;
}

// Scratch of the sort / accumulate stages.  The sort's own buffers (bcnt, btot, bstart, tmp) are
// reused piece after piece on one stream; its outputs (SortOut) and the accumulate's crossing-bucket
// pieces and queues are per piece / per accumulate stream.
struct MsmScratch {
  uint32_t *err, *bcnt, *btot, *bstart, *heavy, *multi, *nheavy, *nmulti;
  uint64_t* tmp;
  G1Xyzz *pfirst, *plast;
};
struct SortOut {
  uint32_t* ent;     // the piece's sorted entries (virtual point | sign << 31)
  uint32_t* gst;     // bucket starts, nbt + 1 (gst[nbt] = the entry total)
  uint32_t* tstart;  // owner bucket of every accumulate chunk
  uint32_t K, T;     // entries per accumulate thread, accumulate threads
};

// Digits + two-level counting sort of points [0, m) (virtual points i and, with GLV, nsplit + i)
// into so, on stream st.  With phix set (bases resident) k_bin_hist also writes the GLV table;
// check_bases: Montgomery bases checked to be reduced on the way.
static int msm_sort(const MsmPlan& p, const MsmScratch& w, const SortOut& so, const G1Aff* bases,
                    const Fr* scalars, size_t m, int mont_in, int device, hipStream_t st, uint4* phix,
                    uint32_t nsplit, int check_bases, hipEvent_t ev_sort_mid, hipStream_t side = nullptr,
                    hipEvent_t ev_fork = nullptr, hipEvent_t ev_join = nullptr, uint32_t w0 = 0,
                    uint32_t nw = 0, uint4* stored = nullptr) {
  const int LOGB = p.c - 1;
  const int nb = p.glv ? 128 : 255;
  const uint32_t CB = (uint32_t)coarse_bits(p.c, nb), FB = (uint32_t)LOGB - CB, NBIN = 1u << CB;
  if (nw == 0) nw = p.W;  // windows [w0, w0 + nw); so's buckets are those windows' (w - w0) * B + b
  const uint32_t nwb = nw * NBIN;
  const uint32_t npts = (uint32_t)m;  // real points (GLV: 2 m virtual ones)
  const uint32_t ep = p.glv ? 2 * p.W : p.W;
  const uint32_t nblk = cdiv(npts, sort_chunk((int)ep));
  // u32 entries when every virtual point index (below nsplit + m with GLV, m without) fits
  const uint64_t vmax = p.glv ? (uint64_t)nsplit + npts : (uint64_t)npts;
  int e32 = vmax <= (uint64_t(1) << (31 - FB)) ? 1 : 0;
  if (const char* e = getenv("SVGPU_SORT_E32")) e32 = e32 && atoi(e) != 0;
  static const int xcd = !getenv("SVGPU_SORT_XCD") || atoi(getenv("SVGPU_SORT_XCD")) != 0 ? 1 : 0;
  // block-major per-block counts + the tiled scan (SVGPU_SORT_BM=0: key-major, k_bin_scan_chunks)
  static const int bm = !getenv("SVGPU_SORT_BM") || atoi(getenv("SVGPU_SORT_BM")) != 0 ? 1 : 0;
  // SVGPU_HIST_PF=0 (read per call): the histogram pass without the one-ahead loads (29-bit table path)
  const int hist_pf = !getenv("SVGPU_HIST_PF") || atoi(getenv("SVGPU_HIST_PF")) != 0;
  SV_LAUNCH_C(k_bin_hist, p.glv, p.c, dim3(nblk), dim3(kBlock), scalars, npts, mont_in, nblk, w.bcnt, w.err, bases,
              phix, p.r29 ? kPhiVtab : p.phi64, check_bases, xcd, bm, w0, nw, stored, hist_pf);
  SV_HIP(hipGetLastError());
  if (ev_sort_mid) SV_HIP(hipEventRecord(ev_sort_mid, st));
  if (bm) {
    // SVGPU_SCAN_KEYS=16: tiles of 16 keys (twice the blocks, 64 row groups per key); default 32
    const char* ke = getenv("SVGPU_SCAN_KEYS");
    if (ke && atoi(ke) == 16)
      hipLaunchKernelGGL(k_bin_scan_tiles<16>, dim3(cdiv(nwb, 16)), dim3(1024), 0, st, w.bcnt, nblk, nwb, w.btot);
    else
      hipLaunchKernelGGL(k_bin_scan_tiles<32>, dim3(cdiv(nwb, 32)), dim3(1024), 0, st, w.bcnt, nblk, nwb, w.btot);
  } else {
    hipLaunchKernelGGL(k_bin_scan_chunks, dim3(nwb), dim3(kBlock), 0, st, w.bcnt, nblk, w.btot);
  }
  // (fusing this scan into k_bin_scan_chunks' last block -- device-scope fence + counter -- was
  // measured 12 -> 122 us for that kernel: the fence writes back the XCD's L2)
  hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, st, w.btot, nwb, w.bstart, so.gst + (size_t)nw * p.B);
  SV_LAUNCH_C(k_bin_scatter, p.glv, p.c, dim3(nblk), dim3(kBlock), scalars, npts, mont_in, nblk, w.bcnt, w.btot, w.bstart,
              w.tmp, e32, xcd, bm, w0, nw, stored);
  static thread_local int fine_attr_dev = -1;  // the > 64 KiB dynamic-LDS opt-in, once per thread/device
  if (fine_attr_dev != device) {
    SV_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fine_sort<0>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFineLds));
    SV_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fine_sort<1>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFineLds));
    SV_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fine_sort<2>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFineLds));
    fine_attr_dev = device;
  }
  // one launch for both region kinds (SVGPU_FINE_SPLIT=1: the round-2 pair of launches, the large
  // regions optionally on a side stream)
  const bool fine_split = getenv("SVGPU_FINE_SPLIT") && atoi(getenv("SVGPU_FINE_SPLIT")) != 0;  // per call
  if (!fine_split && !side) {
    hipLaunchKernelGGL(k_fine_sort<2>, dim3(nwb), dim3(1024), kFineLds, st, w.tmp, e32, w.bstart, FB, so.K, so.gst,
                       so.tstart, so.ent);
    SV_HIP(hipGetLastError());
    return SV_OK;
  }
  // the two instantiations touch disjoint regions: with a side stream the large-region one (a few
  // dozen blocks, the top windows' crowded bins) runs concurrently with the other
  hipStream_t big_st = side ? side : st;
  if (side) {
    SV_HIP(hipEventRecord(ev_fork, st));
    SV_HIP(hipStreamWaitEvent(side, ev_fork, 0));
  }
  hipLaunchKernelGGL(k_fine_sort<1>, dim3(nwb), dim3(1024), kFineLds, big_st, w.tmp, e32, w.bstart, FB, so.K,
                     so.gst, so.tstart, so.ent);
  hipLaunchKernelGGL(k_fine_sort<0>, dim3(nwb), dim3(1024), kFineLds, st, w.tmp, e32, w.bstart, FB, so.K, so.gst,
                     so.tstart, so.ent);
  if (side) {
    SV_HIP(hipEventRecord(ev_join, side));
    SV_HIP(hipStreamWaitEvent(st, ev_join, 0));
  }
  SV_HIP(hipGetLastError());
  return SV_OK;
}

// Bucket accumulation of a sorted piece + its crossing-bucket fixups into bsum, on stream st
// (add_into: the piece's bucket sums are added to what bsum holds -- k_accumulate<true> starts each
// bucket's owner segment from it; otherwise complete buckets are stored and empty ones left alone).
static int msm_acc(const MsmPlan& p, const MsmScratch& w, const SortOut& so, const G1Aff* bases, int add_into,
                   hipStream_t st, G1Xyzz* bsum, const uint4* phix, uint32_t nsplit, hipEvent_t ev_acc_done,
                   hipEvent_t ev_fix_mid, uint32_t nbt = 0) {
  if (nbt == 0) nbt = p.nbt;  // the buckets so covers (a window half: its windows' buckets)
  // (a point prefetch one entry ahead, k_accumulate<., ., 2>, measured no gain on the device path or
  // on the host-fed pieces' ~2 waves per SIMD: 2^20 host-fed 2.69-2.71 ms either way)
  const int r29 = p.r29;
  if (r29) nsplit = ~0u;  // phix is the 29-bit chain's table of every virtual point (vtab_put): record idx
  auto kern = add_into ? (r29 ? k_accumulate<true, true> : k_accumulate<true, false>)
                       : (r29 ? k_accumulate<false, true> : k_accumulate<false, false>);
  hipLaunchKernelGGL(kern, dim3(cdiv(so.T, kBlock)), dim3(kBlock), 0, st, bases, so.ent, so.gst, so.tstart, nbt,
                     so.K, so.T, bsum, w.pfirst, w.plast, w.multi, w.nmulti, w.heavy, w.nheavy, phix, nsplit,
                     p.phi64);
  SV_HIP(hipGetLastError());
  if (ev_acc_done) SV_HIP(hipEventRecord(ev_acc_done, st));
  const uint32_t gm = std::min<uint32_t>(cdiv(nbt, kBlock), 1024);
  hipLaunchKernelGGL(k_fixup, dim3(gm + 256), dim3(kBlock), 0, st, so.gst, so.K, w.pfirst, w.plast, w.multi,
                     w.nmulti, w.heavy, w.nheavy, gm, bsum, r29);
  SV_HIP(hipGetLastError());
  if (ev_fix_mid) SV_HIP(hipEventRecord(ev_fix_mid, st));
  return SV_OK;
}

// Host-fed piece boundaries: SVGPU_H2D_SPLIT = comma-separated weights, else `pieces` equal pieces
// (SVGPU_H2D_PIECES), else the default schedule: 4 equal pieces from 2^18 points.  A piece's
// accumulate runs once its bases have landed (96 B per point at ~52 GB/s), and once the first piece
// is in, the compute stream is the bottleneck (a piece's accumulate + fixup outlasts the next
// piece's transfer), so what counts is the total accumulate work -- smaller pieces are less efficient
// -- against starting early and leaving little after the last byte.  Measured at 2^20 (3 boxes,
// tools/host_api_bench.py): 4 equal pieces 2.73-2.92 ms, 2,2,3,3,3,3 2.74-3.06, 2,3,3,3,3,2
// 2.74-3.09, 3 pieces 3.41-3.47, 6 3.17-4.20 (before per-piece K), 1 piece 3.76-3.95.
static std::vector<size_t> piece_bounds(size_t n, int pieces, const std::vector<double>& dflt) {
  std::vector<double> wts;
  if (const char* e = getenv("SVGPU_H2D_SPLIT")) {
    for (const char* q = e; *q;) {
      char* end = nullptr;
      const double v = strtod(q, &end);
      if (end == q) break;
      if (v > 0) wts.push_back(v);
      q = *end == ',' ? end + 1 : end;
      if (*end && *end != ',') break;
    }
  }
  if (wts.empty()) {
    if (pieces > 0) {
      wts.assign(std::min(pieces, 16), 1.0);
    } else if (n >= (size_t(1) << 18) && !dflt.empty()) {
      wts = dflt;
    } else if (n >= (size_t(1) << 18)) {
      // decreasing: the copy (1.7 ns per point) outpaces the pieces' accumulates (~1.3 ns), so the
      // last piece -- whose accumulate is the call's tail -- is the smallest (round 4, 2^20, three
      // A/B pairs: 5,4,4,3 2.594-2.597 ms vs 4 equal 2.639-2.657; 5,4,4,2,1 2.669-2.670)
      wts = {5, 4, 4, 3};
    } else if (n >= (size_t(1) << 15)) {
      wts = {1, 1};
    } else {
      wts = {1};
    }
  }
  if (wts.size() > 16) wts.resize(16);
  // pieces below 4096 points are not worth a launch sequence
  while (wts.size() > 1 && n < wts.size() * 4096) wts.pop_back();
  double tot = 0;
  for (double v : wts) tot += v;
  std::vector<size_t> b{0};
  double cum = 0;
  for (size_t k = 0; k + 1 < wts.size(); k++) {
    cum += wts[k];
    // boundaries on multiples of 1024 points: every piece's copies start 32-KiB aligned (5 equal
    // pieces, boundaries 32-B aligned, measured 3.13-3.17 ms vs 2.73-2.76 for 4 and 6)
    const size_t at = ((size_t)((double)n * cum / tot)) & ~size_t(1023);
    b.push_back(std::max(b.back(), std::min(n, at)));
  }
  b.push_back(n);
  b.erase(std::unique(b.begin(), b.end()), b.end());
  if (b.size() < 2) b = {0, n};
  return b;
}

static int msm_run_impl(const void* d_bases, const void* d_scalars, size_t n, int form, int device,
                        hipStream_t user_stream, const MsmFeed* feed, host::Xyzz* out) {
  if (n == 0) {
    set_error("pairs should not be empty");
    return SV_ERR_EMPTY;
  }
  if (n > (size_t(1) << 26)) {
    set_error("n = %zu exceeds the per-device limit 2^26 (shard across devices/calls)", n);
    return SV_ERR_LEN;
  }
  if (form != SV_CANONICAL && form != SV_MONTGOMERY) {
    set_error("bad form %d", form);
    return SV_ERR_ARG;
  }
  WsLease lease(device, user_stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  hipStream_t st = ws->stream;
  // Small MSMs (round 5): the window sums on the device, the window Horner on the host
  // (msm_batch_windows_host, msm_batch.hip): the pipeline below is latency-bound there (a 64-term
  // MSM took ~0.35 ms: a dozen launches, serial accumulate chunks, the reduction kernels and a host
  // Horner over 52 windows).  SVGPU_SMALL_MSM=0 keeps the pipeline (read per call).
  if (n <= kSmallMsmTerms && !(getenv("SVGPU_SMALL_MSM") && atoi(getenv("SVGPU_SMALL_MSM")) == 0)) {
    g_last_stats = sv_msm_stats{};
    if (!feed) return msm_batch_windows_host(d_bases, d_scalars, nullptr, 1, n, form, form, device, st, out);
    const size_t sbytes = Workspace::aligned(n * sizeof(Fr));
    SV_TRY(ws->reserve_in(sbytes + n * sizeof(G1Aff)));
    void* ds = ws->inbuf;
    void* db = ws->inbuf + sbytes;
    SV_TRY(feed->stage_scalars(0, n, ds, st, ws->ev[0]));
    SV_TRY(feed->stage_bases(0, n, db, st, ws->ev[1]));
    return msm_batch_windows_host(db, ds, nullptr, 1, n, form, form, device, st, out);
  }
  MsmPlan p = msm_plan(n);
  // host-fed inputs arrive in pieces (piece_bounds): piece k is sorted on the sort stream once its
  // scalars have landed and accumulated on the compute stream once its bases have, while later
  // pieces are still in flight
  const std::vector<size_t> pb = feed ? piece_bounds(n, feed->pieces, feed->split) : std::vector<size_t>{0, n};
  const int pieces = (int)pb.size() - 1;
  const uint32_t ep = p.glv ? 2 * p.W : p.W;  // entries per real point
  size_t max_piece = 0;
  uint64_t tst_total = 0;
  uint32_t Tmax = 0;
  std::vector<SortOut> so(pieces);
  for (int k = 0; k < pieces; k++) {
    const uint64_t e = (uint64_t)(pb[k + 1] - pb[k]) * ep;
    max_piece = std::max(max_piece, pb[k + 1] - pb[k]);
    so[k].K = feed ? piece_K(e, p.nbt) : p.K;  // each piece's chunk length for its own size
    so[k].T = cdiv(e, so[k].K);
    tst_total += (uint64_t)so[k].T + 1;
    Tmax = std::max(Tmax, so[k].T);
  }
  const uint64_t entries = (uint64_t)n * ep;              // all pieces
  const uint64_t piece_entries = (uint64_t)max_piece * ep;  // the sort scratch, reused per piece
  // SVGPU_MSM_SPLIT=1 (device-resident inputs; off by default): the windows in two halves
  // A = [0, WA), B = [WA, W), each sorted, accumulated and reduced on its own, so that half B's sort
  // runs on the sort stream beside half A's accumulate and half A's reduction beside half B's
  // accumulate.  Measured slower at 2^20 (round 4, two A/B pairs: 1.89-1.92 vs 1.81-1.82 ms/step):
  // a half sort costs 0.155 ms, not half of 0.195 (every point's GLV split and digits are still
  // computed), and the two accumulate launches barely overlap (span 1.47 ms, their own durations
  // 1.52 ms): k_accumulate holds two 256-thread blocks per CU, so half A's 512 blocks already fill
  // the chip and half B's wait for them -- one round of blocks each, as the whole launch's two.
  const bool split_env = getenv("SVGPU_MSM_SPLIT") && atoi(getenv("SVGPU_MSM_SPLIT")) != 0;  // per call
  const bool split = !feed && split_env && p.W >= 2 && p.tree == 1 && n >= (size_t(1) << 16);
  const uint32_t nwh[2] = {split ? p.W / 2 : p.W, split ? p.W - p.W / 2 : 0};
  uint32_t Th[2] = {0, 0};
  if (split) {
    for (int h = 0; h < 2; h++) Th[h] = cdiv((uint64_t)p.npts * nwh[h], p.K);
    tst_total = (uint64_t)Th[0] + 1 + Th[1] + 1;
    Tmax = Th[0] + Th[1];
  }

  // ---- workspace layout
  const int nb = p.glv ? 128 : 255;
  const uint32_t CB = (uint32_t)coarse_bits(p.c, nb), NBIN = 1u << CB;
  const uint32_t nwb = p.W * NBIN;
  const uint32_t nblk = cdiv(max_piece, sort_chunk((int)ep));
  size_t bytes = 0;
  auto add = [&](size_t b) { bytes += Workspace::aligned(b); };
  const bool conv = (form == SV_CANONICAL);
  if (conv) add(n * sizeof(G1Aff));
  // GLV: beta x (or phi(P)) per point; the 29-bit chain: its table of every virtual point instead
  const size_t tab4 = p.r29 ? vtab_uint4_per_point(p.glv) : (p.glv ? (p.phi64 ? 4 : 2) : 0);  // uint4 per point
  if (tab4) add(n * tab4 * sizeof(uint4));
  const size_t nfinal = (size_t)p.W * p.NG;
  uint32_t gparts = nfinal < 256 ? 2 : 1;      // k_group_sum blocks per group (see there)
  if (const char* e = getenv("SVGPU_GROUP_P")) gparts = (uint32_t)std::max(1, atoi(e));
  if (gparts > p.J / 2) gparts = p.J / 2;
  const size_t nerr = 64 + nfinal;             // err flag, heavy/multi queue counters, group counters
  add(nerr * 4);
  add((size_t)nwb * nblk * 4);                // bcnt
  add((size_t)nwb * 4);                       // btot
  add(((size_t)nwb + 1) * 4);                 // bstart
  add(piece_entries * 8);                     // tmp (coarse-binned entries)
  // the histogram pass's digits source for the scatter (32 B per point; the device path without
  // window halves only; SVGPU_SORT_HALVES=0, read per call: recomputed by the scatter instead)
  const char* sh_env = getenv("SVGPU_SORT_HALVES");
  const bool keep_halves = !feed && !split && !(sh_env && atoi(sh_env) == 0);
  if (keep_halves) add(n * 32);
  add((((size_t)p.nbt + 1) * pieces + 1) * 4);  // gst per piece (+ 1: two window halves)
  add(entries * 4);                           // ent (every piece's sorted entries)
  add(tst_total * 4);                         // tstart per piece
  const size_t rec_bytes = bucket_rec_bytes(p.r29);  // bucket-sum records (29-bit chain: 144 B)
  add((size_t)Tmax * rec_bytes * 2);          // pfirst, plast
  add((size_t)p.nbt * rec_bytes);             // bsum
  add((size_t)p.nbt * 4);                     // heavy-bucket queue
  add((size_t)p.nbt * 4);                     // multi-thread-bucket queue
  add((size_t)p.J * p.W * sizeof(G1Xyzz) * 2);  // acc_j, T_j
  add(nfinal * sizeof(G1Xyzz));                 // group sums
  add(nfinal * gparts * sizeof(G1Xyzz));        // group slice sums
  const bool group_tree = p.tree != 0;  // see msm_plan
  const size_t ntree = group_tree ? (size_t)p.W * (p.J / kTreeN) * kTreeOut : 0;
  add(ntree * sizeof(G1Xyzz));                  // per-block tree outputs
  SV_TRY(ws->reserve(bytes));
  SV_TRY(ws->reserve_pinned(nfinal * sizeof(G1Xyzz) + 256));
  if (feed) {
    SV_TRY(ws->reserve_in(Workspace::aligned(n * sizeof(G1Aff)) + Workspace::aligned(n * sizeof(Fr))));
    SV_TRY(ws->ensure_copy_stream());
    SV_TRY(ws->ensure_sort_stream());
    d_bases = ws->inbuf;
    d_scalars = ws->inbuf + Workspace::aligned(n * sizeof(G1Aff));
  }

  const G1Aff* bases = reinterpret_cast<const G1Aff*>(d_bases);
  const Fr* scalars = reinterpret_cast<const Fr*>(d_scalars);
  const int mont_in = form == SV_MONTGOMERY ? 1 : 0;
  G1Aff* bases_m = conv ? ws->carve<G1Aff>(n) : nullptr;
  uint4* phix = tab4 ? ws->carve<uint4>(tab4 * n) : nullptr;
  MsmScratch w;
  // the group sums and the error flag / counters share one region: one D2H copy reads both
  G1Xyzz* ping = ws->carve<G1Xyzz>(nfinal + (nerr * 4 + sizeof(G1Xyzz) - 1) / sizeof(G1Xyzz));
  w.err = reinterpret_cast<uint32_t*>(ping + nfinal);
  w.bcnt = ws->carve<uint32_t>((size_t)nwb * nblk);
  w.btot = ws->carve<uint32_t>(nwb);
  w.bstart = ws->carve<uint32_t>((size_t)nwb + 1);
  w.tmp = ws->carve<uint64_t>(piece_entries);
  uint4* stored = keep_halves ? ws->carve<uint4>(2 * n) : nullptr;
  uint32_t* gst_all = ws->carve<uint32_t>(((size_t)p.nbt + 1) * pieces + 1);
  uint32_t* ent_all = ws->carve<uint32_t>(entries);
  uint32_t* tst_all = ws->carve<uint32_t>(tst_total);
  w.pfirst = reinterpret_cast<G1Xyzz*>(ws->carve<uint4>(Tmax * rec_bytes / 16));
  w.plast = reinterpret_cast<G1Xyzz*>(ws->carve<uint4>(Tmax * rec_bytes / 16));
  G1Xyzz* bsum = reinterpret_cast<G1Xyzz*>(ws->carve<uint4>(p.nbt * rec_bytes / 16));
  w.heavy = ws->carve<uint32_t>(p.nbt);
  w.multi = ws->carve<uint32_t>(p.nbt);
  w.nheavy = w.err + 1;  // zeroed with the error flag
  w.nmulti = w.err + 2;
  G1Xyzz* racc = ws->carve<G1Xyzz>((size_t)p.J * p.W);
  G1Xyzz* rtot = ws->carve<G1Xyzz>((size_t)p.J * p.W);
  G1Xyzz* gpart = ws->carve<G1Xyzz>(nfinal * gparts);
  G1Xyzz* tree_out = group_tree ? ws->carve<G1Xyzz>(ntree) : nullptr;
  {
    uint64_t eo = 0, to = 0;
    for (int k = 0; k < pieces; k++) {
      so[k].ent = ent_all + eo;
      so[k].gst = gst_all + (size_t)k * (p.nbt + 1);
      so[k].tstart = tst_all + to;
      eo += (uint64_t)(pb[k + 1] - pb[k]) * ep;
      to += (uint64_t)so[k].T + 1;
    }
  }

  hipEvent_t* ev = ws->ev;
  // each event record between kernels costs ~5.5 us of idle GPU (rocprof trace): the accumulate is
  // always bracketed (bench.py's live roofline), the sort / fixup splits only with SVGPU_MSM_STATS=1
  // SVGPU_MSM_LEAN=1 (read per call): only the accumulate's two events, no sort / reduce split
  static const bool detail_env = getenv("SVGPU_MSM_STATS") && atoi(getenv("SVGPU_MSM_STATS")) != 0;
  const char* lean_env = getenv("SVGPU_MSM_LEAN");
  const bool lean = lean_env && atoi(lean_env) != 0;
  const bool detail = detail_env && !lean;
  const char* fork_env = getenv("SVGPU_SORT_FORK");
  const bool fork_sort = fork_env && atoi(fork_env) != 0;  // off: measured slower (the join delays the accumulate)
  // a host-fed call that fails part-way leaves copies (and sorts) queued on its other streams: drain
  // them before the lease returns the staging buffers to the pool
  struct Drain {
    Workspace* ws;
    bool armed;
    ~Drain() {
      if (armed) (void)ws->quiesce();
    }
  } drain{ws, feed != nullptr || split};
  if (!lean) SV_HIP(hipEventRecord(ev[0], st));
  SV_HIP(hipMemsetAsync(w.err, 0, nerr * 4, st));
  const uint32_t* half_gst[2] = {nullptr, nullptr};  // split: each window half's bucket starts
  if (!feed) {
    if (conv) {
      hipLaunchKernelGGL(k_to_mont_bases, dim3(cdiv(n, kBlock)), dim3(kBlock), 0, st, bases, bases_m, (uint32_t)n,
                         w.err);
      bases = bases_m;
    }
    hipStream_t side = nullptr;
    if (fork_sort) {
      SV_TRY(ws->ensure_copy_stream());  // idle on the device path
      side = ws->copy_stream;
    }
    const uint32_t nsplit = p.glv ? (uint32_t)n : ~0u;
    if (split) {
      SV_TRY(ws->ensure_sort_stream());
      hipStream_t ss = ws->sort_stream;
      SortOut sh[2];
      MsmScratch wh[2] = {w, w};
      for (int h = 0; h < 2; h++) {
        sh[h].K = p.K;
        sh[h].T = Th[h];
        sh[h].ent = ent_all + (h ? (size_t)p.npts * nwh[0] : 0);  // at most npts entries per window
        sh[h].gst = gst_all + (h ? (size_t)nwh[0] * p.B + 1 : 0);
        sh[h].tstart = tst_all + (h ? Th[0] + 1 : 0);
        wh[h].pfirst = rec_at(w.pfirst, h ? Th[0] : 0, p.r29);
        wh[h].plast = rec_at(w.plast, h ? Th[0] : 0, p.r29);
        wh[h].heavy = w.heavy + (h ? nwh[0] * p.B : 0);
        wh[h].multi = w.multi + (h ? nwh[0] * p.B : 0);
        wh[h].nheavy = w.err + 1 + 2 * h;
        wh[h].nmulti = w.err + 2 + 2 * h;
      }
      // half A on the compute stream: sort (with the GLV table and the base check), accumulate
      SV_TRY(msm_sort(p, w, sh[0], bases, scalars, n, mont_in, device, st, phix, nsplit, mont_in,
                      detail ? ev[1] : nullptr, nullptr, nullptr, nullptr, 0, nwh[0]));
      SV_HIP(hipEventRecord(ev[2], st));
      SV_HIP(hipStreamWaitEvent(ss, ev[2], 0));  // the sort scratch is free, the GLV table written
      SV_TRY(msm_acc(p, wh[0], sh[0], bases, 0, st, bsum, phix, nsplit, ev[3], detail ? ev[4] : nullptr,
                     nwh[0] * p.B));
      // half B on the sort stream, beside A's accumulate
      SV_TRY(msm_sort(p, w, sh[1], bases, scalars, n, mont_in, device, ss, nullptr, nsplit, 0, nullptr, nullptr,
                      nullptr, nullptr, nwh[0], nwh[1]));
      SV_HIP(hipEventRecord(ev[62], ss));
      SV_TRY(msm_acc(p, wh[1], sh[1], bases, 0, ss, rec_at(bsum, (size_t)nwh[0] * p.B, p.r29), phix, nsplit, ev[63], nullptr,
                     nwh[1] * p.B));
      SV_HIP(hipEventRecord(ev[8], ss));
      half_gst[0] = sh[0].gst;
      half_gst[1] = sh[1].gst;
    } else {
      SV_TRY(msm_sort(p, w, so[0], bases, scalars, n, mont_in, device, st, phix, nsplit, mont_in,
                      detail ? ev[1] : nullptr, side, ev[60], ev[61], 0, 0, stored));
      SV_HIP(hipEventRecord(ev[2], st));
      SV_TRY(msm_acc(p, w, so[0], bases, 0, st, bsum, phix, nsplit, ev[3], detail ? ev[4] : nullptr));
    }
  } else {
    // Piece k: the copy stream stages its scalars, then its bases (the pageable copy blocks this
    // thread, so the piece's sort is queued in between and runs during the base transfer); the sort
    // stream sorts the piece once its scalars have landed, beside the previous piece's accumulate;
    // the compute stream converts / checks the landed bases, writes the piece's GLV table and
    // accumulates the piece into the one bucket set (identity-initialised; pieces after the first
    // add into it).
    hipStream_t cs = ws->copy_stream, ss = ws->sort_stream;
    const bool prep_on_sort = !getenv("SVGPU_FED_PREP") || atoi(getenv("SVGPU_FED_PREP")) != 0;
    if (pieces > 1) SV_HIP(hipMemsetAsync(bsum, 0, (size_t)p.nbt * rec_bytes, st));
    SV_HIP(hipEventRecord(ev[6], st));
    SV_HIP(hipStreamWaitEvent(cs, ev[6], 0));
    SV_HIP(hipStreamWaitEvent(ss, ev[6], 0));
    // A feeder (the workspace's helper thread) stages the pieces back to back (a pageable copy blocks
    // the thread that issues it: queueing each piece's ~12 launches from that same thread left the
    // copy engine idle ~30 us per burst, rocprof trace); this thread queues a piece's sort /
    // accumulate as soon as the feeder has recorded the piece's events.  staged = stages done (2k + 1: piece k's scalars, 2k + 2: its
    // bases), -1 once the feeder failed.
    // Piece 0's scalars are staged by THIS thread, right after the helper is woken: the helper's
    // wake-up (a condition variable, tens of us) then overlaps that first copy instead of delaying
    // it, and the helper takes over from piece 0's bases (it spins until the scalars are issued, so
    // the copy stream keeps the scalars-then-bases order).
    std::atomic<int> staged{0}, stop{0};
    int feed_rc = SV_OK;
    std::string feed_err;
    SV_TRY(ws->run_helper([&] {
      int rc = SV_OK;
      // the helper thread has no SV_GUARD: an exception here (std::function / vector allocation in
      // the host pool) becomes the call's SV_ERR_DEVICE instead of std::terminate
      try {
        int st0;
        // also leave when the caller stops before staging piece 0 (its copy failed or threw)
        while ((st0 = staged.load(std::memory_order_acquire)) == 0 && !stop.load(std::memory_order_relaxed))
          std::this_thread::yield();
        for (int k = 0; st0 > 0 && k < pieces && !stop.load(std::memory_order_relaxed); k++) {
          const size_t lo = pb[k], hi = pb[k + 1];
          if (k > 0) {
            rc = feed->stage_scalars(lo, hi, const_cast<Fr*>(scalars) + lo, cs, ev[8 + 3 * k]);
            if (rc != SV_OK) break;
            staged.store(2 * k + 1, std::memory_order_release);
          }
          rc = feed->stage_bases(lo, hi, const_cast<G1Aff*>(bases) + lo, cs, ev[9 + 3 * k]);
          if (rc != SV_OK) break;
          staged.store(2 * k + 2, std::memory_order_release);
        }
      } catch (const std::exception& e) {
        set_error("host-fed MSM feeder: %s", e.what());
        rc = SV_ERR_DEVICE;
      } catch (...) {
        set_error("host-fed MSM feeder: unknown exception");
        rc = SV_ERR_DEVICE;
      }
      if (rc != SV_OK) {
        feed_rc = rc;
        feed_err = sv::last_error();
        staged.store(-1, std::memory_order_release);
      }
    }));
    struct Join {  // on every exit: stop the feeder after its current stage, then wait for it
      Workspace* ws;
      std::atomic<int>& stop;
      ~Join() {
        stop.store(1);
        ws->wait_helper();
      }
    } join{ws, stop};
    {
      // an exception leaving stage_scalars (host-pool allocation) unwinds through join, whose stop
      // releases the helper's wait above; SV_GUARD then turns it into the call's error code
      const int rc0 = feed->stage_scalars(pb[0], pb[1], const_cast<Fr*>(scalars) + pb[0], cs, ev[8]);
      if (rc0 != SV_OK) {
        feed_rc = rc0;
        feed_err = sv::last_error();
        staged.store(-1, std::memory_order_release);  // the helper, spinning on it, exits
        return rc0;
      }
      staged.store(1, std::memory_order_release);
    }
    auto wait_stage = [&](int v) -> int {
      int x;
      while ((x = staged.load(std::memory_order_acquire)) >= 0 && x < v) std::this_thread::yield();
      if (x < 0) {
        set_error("%s", feed_err.c_str());
        return feed_rc;
      }
      return SV_OK;
    };
    for (int k = 0; k < pieces; k++) {
      const size_t lo = pb[k], hi = pb[k + 1], m = hi - lo;
      hipEvent_t sc_ready = ev[8 + 3 * k], b_ready = ev[9 + 3 * k], sorted = ev[10 + 3 * k];
      G1Aff* db = const_cast<G1Aff*>(bases) + lo;
      Fr* dsc = const_cast<Fr*>(scalars) + lo;
      // GLV: piece-local virtual points (i, m + i) over the piece's bases and its slice of the table
      const uint32_t nsplit = p.glv ? (uint32_t)m : ~0u;
      uint4* phix_k = tab4 ? phix + tab4 * lo : nullptr;
      SV_TRY(wait_stage(2 * k + 1));
      SV_HIP(hipStreamWaitEvent(ss, sc_ready, 0));
      SV_TRY(msm_sort(p, w, so[k], nullptr, dsc, m, mont_in, device, ss, nullptr, nsplit, 0, nullptr));
      if (!prep_on_sort) SV_HIP(hipEventRecord(sorted, ss));
      SV_TRY(wait_stage(2 * k + 2));
      // the landed bases' preparation (conversion / check / the piece's phi table) runs on the sort
      // stream behind the piece's sort (round 3: off the compute stream, whose back-to-back
      // accumulates are the host-fed path's critical path once the first piece has landed);
      // SVGPU_FED_PREP=0 keeps it on the compute stream
      hipStream_t ps = prep_on_sort ? ss : st;
      SV_HIP(hipStreamWaitEvent(ps, b_ready, 0));
      const G1Aff* pbases = conv ? bases_m + lo : db;
      if (conv)  // canonical bases converted (and checked) once they have landed
        hipLaunchKernelGGL(k_to_mont_bases, dim3(cdiv(m, kBlock)), dim3(kBlock), 0, ps, db, bases_m + lo,
                           (uint32_t)m, w.err);
      if (p.r29)  // the piece's table (29-bit chain) from the landed (converted) bases, checked
        hipLaunchKernelGGL(k_vtab, dim3(cdiv(m, kBlock)), dim3(kBlock), 0, ps, pbases, (uint32_t)m, phix_k,
                           p.glv ? 1 : 0, conv ? nullptr : w.err);
      else if (!p.glv)
        hipLaunchKernelGGL(k_check_bases, dim3(cdiv(m, kBlock)), dim3(kBlock), 0, ps, db, (uint32_t)m, w.err);
      if (!p.r29 && p.glv)  // the piece's phi table from the landed (converted) bases; Montgomery ones checked
        hipLaunchKernelGGL(k_glv_phix, dim3(cdiv(m, kBlock)), dim3(kBlock), 0, ps, pbases, (uint32_t)m, phix_k,
                           p.phi64, conv ? nullptr : w.err);
      SV_HIP(hipGetLastError());
      if (prep_on_sort) SV_HIP(hipEventRecord(sorted, ss));
      SV_HIP(hipStreamWaitEvent(st, sorted, 0));
      if (k == 0) SV_HIP(hipEventRecord(ev[2], st));
      // each piece has its own fixup queue counters (err[1 + 2k], err[2 + 2k], zeroed with the
      // error flag), so no per-piece memset sits between the accumulates
      MsmScratch wk = w;
      wk.nheavy = w.err + 1 + 2 * k;
      wk.nmulti = w.err + 2 + 2 * k;
      SV_TRY(msm_acc(p, wk, so[k], pbases, k > 0 ? 1 : 0, st, bsum, phix_k, nsplit,
                     k == pieces - 1 ? ev[3] : nullptr, nullptr));
    }
  }
  // bucket reduction: running sums over segments of 2^logL buckets, then the subset sums (with
  // several host-fed pieces every bucket of bsum holds a value: no emptiness table).  (Reducing the top windows
  // first to overlap the host Horner with the lower ones was measured slower: each half-size launch
  // of these occupancy-bound kernels takes nearly as long as the whole -- reduce 0.40 -> 0.67 ms.)
  const bool group_quad = !getenv("SVGPU_GROUP_QUAD") || atoi(getenv("SVGPU_GROUP_QUAD")) != 0;
  if (group_tree) {
    static thread_local int tree_attr_dev = -1;  // the > 64 KiB dynamic-LDS opt-in, once per thread/device
    if (tree_attr_dev != device) {
      SV_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wsum_tree<true, false>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)(2 * kTreeRow)));
      SV_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_wsum_tree<true, true>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)(2 * kTreeRow)));
      tree_attr_dev = device;
    }
    // windows [w0, w0 + nw) of the bucket sums xb (starts gs: empty buckets skipped) -> ping rows
    // running sums on the 29-bit chain when the bucket sums are stored in its form
    auto tree_run = p.r29 ? k_wsum_tree<true, true> : k_wsum_tree<true, false>;
    auto reduce_windows = [&](const G1Xyzz* xb, const uint32_t* gs, uint32_t w0, uint32_t nw) {
      if (p.tree == 2)
        hipLaunchKernelGGL(k_wsum_tree<false>, dim3(p.J / kTreeN * nw), dim3(kTreeN), kTreeRow, st, xb, gs, p.B,
                           p.J, 1u, tree_out, p.r29);
      else
        hipLaunchKernelGGL(tree_run, dim3(p.J / kTreeN * nw), dim3(kTreeN), 2 * kTreeRow, st, xb, gs,
                           p.B, p.J, 1u << p.logL, tree_out, p.r29);
      hipLaunchKernelGGL(k_group_fin, dim3(nw * p.NG), dim3(128), 0, st, tree_out, p.J / kTreeN, p.NG,
                         p.tree == 2 ? 1u : 0u, ping + (size_t)w0 * p.NG);
    };
    if (split) {
      reduce_windows(bsum, half_gst[0], 0, nwh[0]);  // beside half B's accumulate
      SV_HIP(hipStreamWaitEvent(st, ev[8], 0));
      reduce_windows(rec_at(bsum, (size_t)nwh[0] * p.B, p.r29), half_gst[1], nwh[0], nwh[1]);
    } else {
      reduce_windows(bsum, pieces > 1 ? nullptr : so[0].gst, 0, p.W);
    }
  } else {
    hipLaunchKernelGGL(k_wsum, dim3(cdiv((uint64_t)p.J * p.W, kBlock)), dim3(kBlock), 0, st, bsum,
                       pieces > 1 ? nullptr : so[0].gst, p.B, p.J, 1u << p.logL, p.W, 1, racc, rtot, p.r29);
    if (group_quad)
      hipLaunchKernelGGL(k_group_sum_q, dim3(p.NG * p.W * gparts), dim3(kGroupBlock), 0, st, racc, rtot, p.J,
                         p.logJ, gparts, ping, gpart, w.err + 64);
    else
      hipLaunchKernelGGL(k_group_sum, dim3(p.NG * p.W * gparts), dim3(kGroupBlock), 0, st, racc, rtot, p.J,
                         p.logJ, gparts, ping, gpart, w.err + 64);
  }
  SV_HIP(hipGetLastError());
  if (!lean) SV_HIP(hipEventRecord(ev[5], st));
  SV_HIP(hipMemcpyAsync(ws->pinned, ping, nfinal * sizeof(G1Xyzz) + 4, hipMemcpyDeviceToHost, st));
  SV_HIP(hipStreamSynchronize(st));
  drain.armed = false;  // the copy and sort streams' work all precedes the compute stream's end
  uint32_t errv;
  memcpy(&errv, ws->pinned + nfinal * sizeof(G1Xyzz), 4);
  if (errv) {
    set_error("invalid input: %s%s", (errv & 1) ? "base coordinate not reduced mod p; " : "",
              (errv & 2) ? "scalar not reduced mod r" : "");
    return SV_ERR_ARG;
  }
  auto t0 = std::chrono::steady_clock::now();
  *out = host_combine(p, reinterpret_cast<const host::Xyzz*>(ws->pinned));
  auto t1 = std::chrono::steady_clock::now();

  sv_msm_stats& s = g_last_stats;
  float ms = 0;
  if (detail && !feed) {
    (void)hipEventElapsedTime(&ms, ev[0], ev[1]);
    s.digits_ms = ms;  // digits + coarse histogram (digits never stored; the GLV halves are)
    (void)hipEventElapsedTime(&ms, ev[1], ev[2]);
    s.sort_ms = ms;
    (void)hipEventElapsedTime(&ms, ev[3], ev[4]);
    s.fixup_ms = ms;
    (void)hipEventElapsedTime(&ms, ev[4], ev[5]);
    s.reduce_ms = ms;
  } else if (lean) {
    s.digits_ms = s.sort_ms = s.fixup_ms = s.reduce_ms = -1.0f;  // not measured
  } else {  // digits folded into sort_ms, fixup into reduce_ms
    s.digits_ms = 0;
    (void)hipEventElapsedTime(&ms, ev[0], ev[2]);
    s.sort_ms = ms;
    s.fixup_ms = 0;
    (void)hipEventElapsedTime(&ms, ev[3], ev[5]);
    s.reduce_ms = ms;
  }
  // host-fed: "accumulate" spans the first piece's accumulate to the last piece's (transfers included);
  // split: the two halves' accumulate launches, each from its own start to its own end (they may
  // overlap in time), and accumulate_span_ms from the first start to the last end
  (void)hipEventElapsedTime(&ms, ev[2], ev[3]);
  s.accumulate_ms = ms;
  s.accumulate_span_ms = ms;
  s.accumulate_launches = 1;
  if (split) {
    float mb = 0, mspan = 0;
    (void)hipEventElapsedTime(&mb, ev[62], ev[63]);
    (void)hipEventElapsedTime(&mspan, ev[2], ev[63]);
    s.accumulate_ms = ms + mb;
    s.accumulate_span_ms = std::max(ms, mspan);
    s.accumulate_launches = 2;
  }
  s.host_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
  if (lean) {
    s.total_ms = -1.0f;
  } else {
    (void)hipEventElapsedTime(&ms, ev[0], ev[5]);
    s.total_ms = ms + s.host_ms;
  }
  s.window_bits = p.c;
  s.num_windows = p.W;
  s.accumulate_launch_units = cdiv((uint64_t)p.npts * p.W, p.K);
  s.entries = (uint64_t)p.npts * p.W;
  return SV_OK;
}

int msm_run_device(const void* d_bases, const void* d_scalars, size_t n, int form, int device,
                   hipStream_t user_stream, host::Xyzz* out) {
  return msm_run_impl(d_bases, d_scalars, n, form, device, user_stream, nullptr, out);
}

int msm_run_fed(size_t n, int form, int device, const MsmFeed& feed, host::Xyzz* out) {
  return msm_run_impl(nullptr, nullptr, n, form, device, nullptr, &feed, out);
}

}  // namespace sv
