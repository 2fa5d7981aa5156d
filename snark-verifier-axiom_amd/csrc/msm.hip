// Pippenger bucket MSM for BN254 G1 on gfx950.
//
// Replaces util::msm::multi_scalar_multiplication (snark-verifier/src/util/msm.rs:238-316) and
// the naive NativeLoader::multi_scalar_multiplication (snark-verifier/src/loader/native.rs:61-71):
// same group element out, computed as a signed-digit bucket method.
//
// Pipeline (all on one stream, inputs already in HBM):
//   k_to_mont_bases   (canonical input only) bases -> Montgomery workspace copy
//   k_bin_hist        per block of 2048 points: signed c-bit digits of every window (never
//                     stored), LDS histogram of (window, coarse bin = top bits of the bucket)
//   k_bin_scan_chunks / k_bin_scan   offsets of every (window, bin, block) run
//   k_bin_scatter     digits again; entries appended to their block's (window, bin) run -> tmp
//   k_fine_sort       one block per (window, bin): counting sort by the fine bucket index inside
//                     the bin's L2-resident region -> ent[], bucket offsets gst[], owner bucket of
//                     every accumulate chunk tstart[]
//   k_accumulate      each thread sums K consecutive sorted entries (mixed XYZZ adds; perfect
//                     load balance whatever the digit distribution), complete buckets written
//                     directly, bucket pieces that cross a thread boundary to pfirst/plast
//   k_fixup           per bucket: join the pieces of buckets that cross thread boundaries
//   k_wsum            bucket reduction, step 1: F_w = sum_b (b+1) S_b = sum_j acc_j + L sum_j j T_j
//                     with running sums over segments of L = 8 buckets (acc_j, T_j per segment)
//   k_group_sum       step 2: sum_j j T_j = sum_k 2^k U_k, U_k = sum_{j : bit k of j} T_j; the
//                     subset sums U_k and the plain sum of acc_j are independent, so each is one
//                     block-level tree reduction in LDS (low serial depth: the tail is latency-bound)
//   host              Horner over (window, bit) terms (~255 doublings) -> affine, see host_ec.hpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "curve.hpp"
#include "host_ec.hpp"
#include "msm.hpp"
#include "runtime.hpp"

namespace sv {

static constexpr int kBlock = 256;

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

// Signed windows: digit_w = bits[cw, cw+c) + carry, mapped to (-2^(c-1), 2^(c-1)].  W = ceil(255/c)
// windows so the top digit never carries out (scalars < r < 2^254).  f(w, mag, neg) per window.
template <int C, class F>
__device__ __forceinline__ void for_each_digit(const Fr& s, F&& f) {
  constexpr int W = (255 + C - 1) / C;
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

// ---- two-level counting sort of the n * W (point, digit) entries by bucket ------------------
// Bucket b = |digit| - 1 of window w splits into a coarse bin b >> FB (NBIN = 2^CB bins per window)
// and a fine index b & (2^FB - 1).  Pass 1 (k_bin_hist): per block of sort_chunk(c) points, every
// window's digits, LDS histogram of (window, bin).  Pass 2 (k_bin_scan_chunks, k_bin_scan): global
// offsets of every (window, bin, block) run.  Pass 3 (k_bin_scatter): the digits again, each
// entry appended to its block's run -> tmp (u64: fine << 32 | point | sign << 31); a block's runs
// are short contiguous spans, so writes merge in L2.  Pass 4 (k_fine_sort): one block per
// (window, bin) counting-sorts its ~n / NBIN entries by fine index inside that bin's region (L2
// resident), writes ent[], the global bucket offsets gst[] and the owner bucket tstart[t] of every
// accumulate chunk [tK, tK + K).  No per-(window, point) digit array is ever stored.
// points per block in passes 1 and 3: 512 (2 per thread), 256 when the LDS staging of W digits
// per point would not fit (small c, many windows)
__host__ __device__ constexpr uint32_t sort_chunk(int c) { return (255 + c - 1) / c > 20 ? 256u : 512u; }

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

template <int C>
__global__ void __launch_bounds__(kBlock) k_bin_hist(const Fr* __restrict__ scalars, uint32_t n, int mont_in,
                                                     uint32_t nblk, uint32_t* __restrict__ bcnt,
                                                     uint32_t* __restrict__ err) {
  constexpr int W = (255 + C - 1) / C, LOGB = C - 1;
  constexpr int CB = LOGB < 6 ? LOGB : 6, FB = LOGB - CB, NBIN = 1 << CB;
  __shared__ uint32_t h[W * NBIN];
  for (int k = threadIdx.x; k < W * NBIN; k += kBlock) h[k] = 0;
  __syncthreads();
  constexpr uint32_t CH = sort_chunk(C);
  const uint32_t lo = blockIdx.x * CH, hi = min(n, lo + CH);
  for (uint32_t i = lo + threadIdx.x; i < hi; i += kBlock) {
    const Fr s = load_scalar(scalars, i, mont_in, err);
    for_each_digit<C>(s, [&](int w, uint32_t mag, uint32_t) {
      if (mag) atomicAdd(&h[w * NBIN + ((mag - 1) >> FB)], 1u);
    });
  }
  __syncthreads();
  // layout bcnt[(w * NBIN + bin) * nblk + blk]: each (window, bin) scans over contiguous blocks
  for (int k = threadIdx.x; k < W * NBIN; k += kBlock) bcnt[(size_t)k * nblk + blockIdx.x] = h[k];
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

// one 1024-thread block: exclusive scan of btot over all (window, bin) -> bstart; bstart[nwb] = total
__global__ void __launch_bounds__(1024) k_bin_scan(const uint32_t* __restrict__ btot, uint32_t nwb,
                                                   uint32_t* __restrict__ bstart) {
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
  if (tid == 1023) bstart[nwb] = part[1023];
}

// Pass 3: the block's entries are first placed in LDS grouped by (window, bin), then each group
// is copied to its global run with consecutive lanes writing consecutive addresses.
template <int C>
__global__ void __launch_bounds__(kBlock) k_bin_scatter(const Fr* __restrict__ scalars, uint32_t n, int mont_in,
                                                        uint32_t nblk, const uint32_t* __restrict__ bcnt,
                                                        const uint32_t* __restrict__ bstart,
                                                        uint64_t* __restrict__ tmp) {
  constexpr int W = (255 + C - 1) / C, LOGB = C - 1;
  constexpr int CB = LOGB < 6 ? LOGB : 6, FB = LOGB - CB, NBIN = 1 << CB, NK = W * NBIN;
  constexpr uint32_t FMASK = (1u << FB) - 1;
  constexpr uint32_t CH = sort_chunk(C), PT = CH / kBlock;
  __shared__ uint32_t off[NK];   // local group offsets
  __shared__ uint32_t cur[NK];   // cursors
  __shared__ uint32_t part[kBlock];
  __shared__ uint32_t stage[CH * W];  // local point (9 bits) | sign << 9 | fine << 10
  __shared__ uint16_t key[CH * W];
  const uint32_t blk = blockIdx.x, lo = blk * CH, hi = min(n, lo + CH);
  for (int k = threadIdx.x; k < NK; k += kBlock) off[k] = 0;
  __syncthreads();
  Fr sc[PT];
#pragma unroll
  for (int j = 0; j < (int)PT; j++) {
    const uint32_t i = lo + threadIdx.x + j * kBlock;
    if (i < hi) {
      sc[j] = load_scalar(scalars, i, mont_in, nullptr);
      for_each_digit<C>(sc[j], [&](int w, uint32_t mag, uint32_t) {
        if (mag) atomicAdd(&off[w * NBIN + ((mag - 1) >> FB)], 1u);
      });
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
      for_each_digit<C>(sc[j], [&](int w, uint32_t mag, uint32_t neg) {
        if (mag) {
          const uint32_t b = mag - 1;
          const uint32_t k = w * NBIN + (b >> FB);
          const uint32_t pos = atomicAdd(&cur[k], 1u);
          stage[pos] = li | (neg << 9) | ((b & FMASK) << 10);
          key[pos] = (uint16_t)k;
        }
      });
    }
  }
  __syncthreads();
  // global position of local slot x = gbase[key] + x  (cur[] reused for gbase)
  for (int k = threadIdx.x; k < NK; k += kBlock) cur[k] = bstart[k] + bcnt[(size_t)k * nblk + blk] - off[k];
  __syncthreads();
  for (uint32_t x = threadIdx.x; x < total; x += kBlock) {
    const uint32_t e = stage[x];
    tmp[cur[key[x]] + x] = ((uint64_t)(e >> 10) << 32) | (lo + (e & 511u)) | (((e >> 9) & 1u) << 31);
  }
}

// one block per (window, bin): counting sort by the fine index within the bin's region
__global__ void __launch_bounds__(1024) k_fine_sort(const uint64_t* __restrict__ tmp,
                                                    const uint32_t* __restrict__ bstart, uint32_t FB, uint32_t K,
                                                    uint32_t* __restrict__ gst, uint32_t* __restrict__ tstart,
                                                    uint32_t* __restrict__ ent) {
  __shared__ uint32_t fc[512];
  __shared__ uint32_t part[1024];
  const uint32_t wb = blockIdx.x, tid = threadIdx.x, NF = 1u << FB;
  const uint32_t s0 = bstart[wb], s1 = bstart[wb + 1];
  for (uint32_t f = tid; f < NF; f += 1024) fc[f] = 0;
  __syncthreads();
  {
    uint32_t e = s0 + tid;
    for (; e + 3 * 1024 < s1; e += 4 * 1024) {  // 4 loads in flight per thread
      const uint32_t f0 = (uint32_t)(tmp[e] >> 32), f1 = (uint32_t)(tmp[e + 1024] >> 32);
      const uint32_t f2 = (uint32_t)(tmp[e + 2048] >> 32), f3 = (uint32_t)(tmp[e + 3072] >> 32);
      atomicAdd(&fc[f0], 1u);
      atomicAdd(&fc[f1], 1u);
      atomicAdd(&fc[f2], 1u);
      atomicAdd(&fc[f3], 1u);
    }
    for (; e < s1; e += 1024) atomicAdd(&fc[(uint32_t)(tmp[e] >> 32)], 1u);
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
    fc[tid] = st;
    for (uint32_t t = (st + K - 1) / K; t * K < en; t++) tstart[t] = g;
  }
  __syncthreads();
  uint32_t e = s0 + tid;
  for (; e + 3 * 1024 < s1; e += 4 * 1024) {
    uint64_t x[4];
#pragma unroll
    for (int j = 0; j < 4; j++) x[j] = tmp[e + j * 1024];
#pragma unroll
    for (int j = 0; j < 4; j++) ent[atomicAdd(&fc[(uint32_t)(x[j] >> 32)], 1u)] = (uint32_t)x[j];
  }
  for (; e < s1; e += 1024) {
    const uint64_t x = tmp[e];
    ent[atomicAdd(&fc[(uint32_t)(x >> 32)], 1u)] = (uint32_t)x;
  }
}

// Each thread: K consecutive sorted entries.  See file header.
__global__ void __launch_bounds__(kBlock) k_accumulate(
    const G1Aff* __restrict__ bases, const uint32_t* __restrict__ ent, const uint32_t* __restrict__ gst,
    const uint32_t* __restrict__ tstart, uint32_t nbt, uint32_t K, uint32_t T,
    G1Xyzz* __restrict__ bsum, G1Xyzz* __restrict__ pfirst, G1Xyzz* __restrict__ plast) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const uint32_t m = gst[nbt];
  const uint32_t s0 = t * K;
  if (s0 >= m) return;
  const uint32_t e_end = min(s0 + K, m);
  uint32_t g = tstart[t];
  uint32_t gs = gst[g], ge = gst[g + 1];
  uint32_t seg_start = s0;
  bool first = true;
  G1Xyzz acc = G1Xyzz::identity();
  for (uint32_t e = s0; e < e_end; e++) {
    if (e >= ge) {
      if (seg_start == gs && e == ge) store_xyzz(bsum, g, acc);
      else if (first) store_xyzz(pfirst, t, acc);
      else store_xyzz(plast, t, acc);
      first = false;
      do {
        g++;
        gs = ge;
        ge = gst[g + 1];
      } while (ge <= e);
      seg_start = e;
      acc = G1Xyzz::identity();
    }
    uint32_t v = ent[e];
    G1Aff p = load_aff(bases, v & 0x7fffffffu);
    if (v & 0x80000000u) p.y = -p.y;
    acc = xyzz_madd_aff(acc, p);
  }
  if (seg_start == gs && e_end == ge) store_xyzz(bsum, g, acc);
  else if (first) store_xyzz(pfirst, t, acc);
  else store_xyzz(plast, t, acc);
}

// Per global bucket: empty -> identity; crossing thread boundaries -> join the pieces.  A bucket
// spanning more than kFixSerial threads (skewed digits: all-equal scalars, a short top window) is
// queued for k_fixup_heavy instead of being walked serially.
static constexpr uint32_t kFixSerial = 8;
__global__ void __launch_bounds__(kBlock) k_fixup(const uint32_t* __restrict__ gst, uint32_t nbt, uint32_t K,
                                                  const G1Xyzz* __restrict__ pfirst, const G1Xyzz* __restrict__ plast,
                                                  G1Xyzz* __restrict__ bsum, uint32_t* __restrict__ heavy,
                                                  uint32_t* __restrict__ nheavy) {
  uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nbt) return;
  uint32_t s = gst[g], e = gst[g + 1];
  if (s == e) {
    store_xyzz(bsum, g, G1Xyzz::identity());
    return;
  }
  uint32_t t0 = s / K, t1 = (e - 1) / K;
  if (t0 == t1) return;
  if (t1 - t0 > kFixSerial) {
    heavy[atomicAdd(nheavy, 1u)] = g;
    return;
  }
  G1Xyzz acc = (s == t0 * K) ? load_xyzz(pfirst, t0) : load_xyzz(plast, t0);
  for (uint32_t t = t0 + 1; t <= t1; t++) acc = xyzz_add(acc, load_xyzz(pfirst, t));
  store_xyzz(bsum, g, acc);
}

// Heavy buckets: one block per queued bucket (grid-stride over the queue), strided partial sums of
// the per-thread pieces + LDS tree.
__global__ void __launch_bounds__(kBlock) k_fixup_heavy(const uint32_t* __restrict__ gst, uint32_t K,
                                                        const G1Xyzz* __restrict__ pfirst,
                                                        const G1Xyzz* __restrict__ plast,
                                                        const uint32_t* __restrict__ heavy,
                                                        const uint32_t* __restrict__ nheavy,
                                                        G1Xyzz* __restrict__ bsum) {
  __shared__ G1Xyzz sh[kBlock];
  const uint32_t nh = *nheavy, tid = threadIdx.x;
  for (uint32_t h = blockIdx.x; h < nh; h += gridDim.x) {
    const uint32_t g = heavy[h];
    const uint32_t s = gst[g], e = gst[g + 1];
    const uint32_t t0 = s / K, t1 = (e - 1) / K;
    G1Xyzz acc = G1Xyzz::identity();
    for (uint32_t t = t0 + 1 + tid; t <= t1; t += kBlock) acc = xyzz_add(acc, load_xyzz(pfirst, t));
    sh[tid] = acc;
    __syncthreads();
    for (uint32_t st = kBlock / 2; st > 0; st >>= 1) {
      if (tid < st) sh[tid] = xyzz_add(sh[tid], sh[tid + st]);
      __syncthreads();
    }
    if (tid == 0) {
      G1Xyzz head = (s == t0 * K) ? load_xyzz(pfirst, t0) : load_xyzz(plast, t0);
      store_xyzz(bsum, g, xyzz_add(head, sh[0]));
    }
    __syncthreads();
  }
}

// One bucket-reduction level over `groups` groups of N elements, segments of L buckets:
//   acc[g][j] = sum_{i in seg j} (i - jL + base) X[g][i],  tot[g][j] = sum_{i in seg j} X[g][i]
__global__ void __launch_bounds__(kBlock) k_wsum(const G1Xyzz* __restrict__ X, uint32_t N, uint32_t J, uint32_t L, uint32_t groups, int base,
                       G1Xyzz* __restrict__ acc_out, G1Xyzz* __restrict__ tot_out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= J * groups) return;
  uint32_t g = tid / J, j = tid % J;
  const G1Xyzz* x = X + (size_t)g * N;
  uint32_t lo = j * L;
  uint32_t hi = min(N, lo + L);
  G1Xyzz run = G1Xyzz::identity(), acc = G1Xyzz::identity();
  for (uint32_t i = hi; i-- > lo;) {
    run = xyzz_add(run, load_xyzz(x, i));
    if (base || i > lo) acc = xyzz_add(acc, run);
  }
  store_xyzz(acc_out, tid, acc);
  if (tot_out) store_xyzz(tot_out, tid, run);
}

// Step 2 fused: one 512-thread block per (window, group) sums the group's H members (strided,
// ~H/512 serial adds per thread) and finishes with an LDS tree (9 levels) -> out[w*NG + q].
static constexpr int kGroupBlock = 512;
__global__ void __launch_bounds__(kGroupBlock) k_group_sum(const G1Xyzz* __restrict__ acc,
                                                           const G1Xyzz* __restrict__ tot, uint32_t J,
                                                           uint32_t logJ, G1Xyzz* __restrict__ out) {
  __shared__ G1Xyzz sh[kGroupBlock];
  const uint32_t NG = 2 + logJ, H = J / 2;
  const uint32_t gid = blockIdx.x, w = gid / NG, q = gid % NG, tid = threadIdx.x;
  G1Xyzz s = G1Xyzz::identity();
  for (uint32_t m = tid; m < H; m += kGroupBlock) {
    G1Xyzz x;
    if (q < 2) {
      x = load_xyzz(acc, w * J + q * H + m);
    } else {
      const uint32_t k = q - 2;
      const uint32_t j = ((m >> k) << (k + 1)) | (1u << k) | (m & ((1u << k) - 1));
      x = load_xyzz(tot, w * J + j);
    }
    s = xyzz_add(s, x);
  }
  sh[tid] = s;
  __syncthreads();
  for (uint32_t st = kGroupBlock / 2; st > 0; st >>= 1) {
    if (tid < st) sh[tid] = xyzz_add(sh[tid], sh[tid + st]);
    __syncthreads();
  }
  if (tid == 0) store_xyzz(out, gid, sh[0]);
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

MsmPlan msm_plan(size_t n) {
  MsmPlan p;
  int lg = 0;
  while ((size_t(1) << (lg + 1)) <= n) lg++;
  int c = lg - 4;
  if (const char* e = getenv("SVGPU_WINDOW_BITS")) c = atoi(e);
  if (c < 4) c = 4;
  if (c > 16) c = 16;
  p.c = c;
  p.W = (255 + c - 1) / c;
  p.B = 1u << (c - 1);
  p.nbt = p.B * p.W;
  uint64_t entries = (uint64_t)n * p.W;
  uint64_t K = entries / (1u << 18);
  if (K < 4) K = 4;
  if (K > 32) K = 32;
  // large n: buckets average entries / nbt >> 32 entries; keep a bucket within ~2-3 threads so the
  // fixup stays a short serial join (a 2^24 MSM at c = 16 has 512 entries per bucket)
  const uint64_t half_bucket = entries / p.nbt / 2;
  if (K < half_bucket) K = half_bucket < 512 ? half_bucket : 512;
  if (const char* e = getenv("SVGPU_ACC_K")) K = (uint64_t)atoi(e);
  if (K < 1) K = 1;
  p.K = (uint32_t)K;
  p.T = cdiv(entries, p.K);
  // reduction: J running-sum segments per window, NG subset groups of H = J/2 points
  p.logL = 3;  // 8 buckets per running-sum segment (swept: tools/gpu_sweep_red.sh)
  if (const char* e = getenv("SVGPU_RED_LOG")) p.logL = atoi(e);
  if (p.logL < 1) p.logL = 1;
  if (p.logL > p.c - 3) p.logL = p.c - 3 > 1 ? p.c - 3 : 1;
  p.J = p.B >> p.logL;
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

#define SV_LAUNCH_C(KERNEL, C, GRID, BLOCK, ...)                                \
  switch (C) {                                                                 \
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
    case 16: hipLaunchKernelGGL(KERNEL<16>, GRID, BLOCK, 0, st, __VA_ARGS__); break; \
    default: break;                                                            \
  }

// Host Horner over (window, group) terms: total = sum_w 2^(c w) [A_lo + A_hi + sum_k 2^(2+k) U_k].
static host::Xyzz host_combine(const MsmPlan& p, const host::Xyzz* A /* [W][NG] */) {
  int maxe = (int)(p.c * (p.W - 1) + p.logL + p.logJ);
  std::vector<host::Xyzz> byexp(maxe + 1, host::x_identity());
  for (uint32_t w = 0; w < p.W; w++)
    for (uint32_t q = 0; q < p.NG; q++) {
      int e = (int)(p.c * w + (q < 2 ? 0 : p.logL + (q - 2)));
      byexp[e] = host::x_add(byexp[e], A[w * p.NG + q]);
    }
  host::Xyzz acc = host::x_identity();
  for (int e = maxe; e >= 0; e--) {
    acc = host::x_dbl(acc);
    acc = host::x_add(acc, byexp[e]);
  }
  return acc;
}

int msm_run_device(const void* d_bases, const void* d_scalars, size_t n, int form, int device,
                   hipStream_t user_stream, host::Xyzz* out) {
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
  const MsmPlan p = msm_plan(n);
  const uint64_t entries = (uint64_t)n * p.W;

  // ---- workspace layout
  const int LOGB = p.c - 1;
  const uint32_t CB = LOGB < 6 ? (uint32_t)LOGB : 6u, FB = (uint32_t)LOGB - CB, NBIN = 1u << CB;
  const uint32_t nwb = p.W * NBIN;
  const uint32_t nblk = cdiv(n, sort_chunk(p.c));
  size_t bytes = 0;
  auto add = [&](size_t b) { bytes += Workspace::aligned(b); };
  bool conv = (form == SV_CANONICAL);
  if (conv) add(n * sizeof(G1Aff));
  add(256);                                   // err flag + heavy-queue counter
  add((size_t)nwb * nblk * 4);                // bcnt
  add((size_t)nwb * 4);                       // btot
  add(((size_t)nwb + 1) * 4);                 // bstart
  add(entries * 8);                           // tmp (coarse-binned entries)
  add(((size_t)p.nbt + 1) * 4);               // gst
  add(entries * 4);                           // ent
  add(((size_t)p.T + 1) * 4);                 // tstart
  add((size_t)p.T * sizeof(G1Xyzz) * 2);      // pfirst, plast
  add((size_t)p.nbt * sizeof(G1Xyzz));        // bsum
  add((size_t)p.nbt * 4);                     // heavy-bucket queue
  const size_t nfinal = (size_t)p.W * p.NG;
  add((size_t)p.J * p.W * sizeof(G1Xyzz) * 2);  // acc_j, T_j
  add(nfinal * sizeof(G1Xyzz));                 // group sums
  SV_TRY(ws->reserve(bytes));
  SV_TRY(ws->reserve_pinned(nfinal * sizeof(G1Xyzz) + 256));

  const G1Aff* bases = reinterpret_cast<const G1Aff*>(d_bases);
  const Fr* scalars = reinterpret_cast<const Fr*>(d_scalars);
  const int mont_in = form == SV_MONTGOMERY ? 1 : 0;
  G1Aff* bases_m = conv ? ws->carve<G1Aff>(n) : nullptr;
  uint32_t* err = ws->carve<uint32_t>(64);
  uint32_t* bcnt = ws->carve<uint32_t>((size_t)nwb * nblk);
  uint32_t* btot = ws->carve<uint32_t>(nwb);
  uint32_t* bstart = ws->carve<uint32_t>((size_t)nwb + 1);
  uint64_t* tmp = ws->carve<uint64_t>(entries);
  uint32_t* gst = ws->carve<uint32_t>((size_t)p.nbt + 1);
  uint32_t* ent = ws->carve<uint32_t>(entries);
  uint32_t* tstart = ws->carve<uint32_t>((size_t)p.T + 1);
  G1Xyzz* pfirst = ws->carve<G1Xyzz>(p.T);
  G1Xyzz* plast = ws->carve<G1Xyzz>(p.T);
  G1Xyzz* bsum = ws->carve<G1Xyzz>(p.nbt);
  uint32_t* heavy = ws->carve<uint32_t>(p.nbt);
  uint32_t* nheavy = err + 1;  // zeroed with the error flag
  G1Xyzz* racc = ws->carve<G1Xyzz>((size_t)p.J * p.W);
  G1Xyzz* rtot = ws->carve<G1Xyzz>((size_t)p.J * p.W);
  G1Xyzz* ping = ws->carve<G1Xyzz>(nfinal);

  hipEvent_t* ev = ws->ev;
  SV_HIP(hipEventRecord(ev[0], st));
  SV_HIP(hipMemsetAsync(err, 0, 256, st));
  if (conv) {
    hipLaunchKernelGGL(k_to_mont_bases, dim3(cdiv(n, kBlock)), dim3(kBlock), 0, st,
                       bases, bases_m, (uint32_t)n, err);
    bases = bases_m;
  }
  SV_LAUNCH_C(k_bin_hist, p.c, dim3(nblk), dim3(kBlock), scalars, (uint32_t)n, mont_in, nblk, bcnt, err);
  SV_HIP(hipGetLastError());
  SV_HIP(hipEventRecord(ev[1], st));
  hipLaunchKernelGGL(k_bin_scan_chunks, dim3(nwb), dim3(kBlock), 0, st, bcnt, nblk, btot);
  hipLaunchKernelGGL(k_bin_scan, dim3(1), dim3(1024), 0, st, btot, nwb, bstart);
  SV_LAUNCH_C(k_bin_scatter, p.c, dim3(nblk), dim3(kBlock), scalars, (uint32_t)n, mont_in, nblk, bcnt, bstart,
              tmp);
  hipLaunchKernelGGL(k_fine_sort, dim3(nwb), dim3(1024), 0, st, tmp, bstart, FB, p.K, gst, tstart, ent);
  SV_HIP(hipMemcpyAsync(gst + p.nbt, bstart + nwb, 4, hipMemcpyDeviceToDevice, st));
  SV_HIP(hipGetLastError());
  SV_HIP(hipEventRecord(ev[2], st));
  hipLaunchKernelGGL(k_accumulate, dim3(cdiv(p.T, kBlock)), dim3(kBlock), 0, st, bases, ent, gst,
                     tstart, p.nbt, p.K, p.T, bsum, pfirst, plast);
  SV_HIP(hipGetLastError());
  SV_HIP(hipEventRecord(ev[3], st));
  hipLaunchKernelGGL(k_fixup, dim3(cdiv(p.nbt, kBlock)), dim3(kBlock), 0, st, gst, p.nbt, p.K, pfirst,
                     plast, bsum, heavy, nheavy);
  hipLaunchKernelGGL(k_fixup_heavy, dim3(256), dim3(kBlock), 0, st, gst, p.K, pfirst, plast, heavy, nheavy,
                     bsum);
  SV_HIP(hipEventRecord(ev[4], st));
  // bucket reduction: running sums over segments of 2^logL buckets, then the subset sums
  hipLaunchKernelGGL(k_wsum, dim3(cdiv((uint64_t)p.J * p.W, kBlock)), dim3(kBlock), 0, st, bsum, p.B, p.J,
                     1u << p.logL, p.W, 1, racc, rtot);
  hipLaunchKernelGGL(k_group_sum, dim3(p.NG * p.W), dim3(kGroupBlock), 0, st, racc, rtot, p.J, p.logJ, ping);
  SV_HIP(hipGetLastError());
  SV_HIP(hipEventRecord(ev[5], st));
  SV_HIP(hipMemcpyAsync(ws->pinned, ping, nfinal * sizeof(G1Xyzz), hipMemcpyDeviceToHost, st));
  SV_HIP(hipMemcpyAsync(ws->pinned + nfinal * sizeof(G1Xyzz), err, 4, hipMemcpyDeviceToHost, st));
  SV_HIP(hipStreamSynchronize(st));
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
  float ms;
  hipEventElapsedTime(&ms, ev[0], ev[1]);
  s.digits_ms = ms;  // digits + coarse histogram (digits are recomputed, never stored)
  hipEventElapsedTime(&ms, ev[1], ev[2]);
  s.sort_ms = ms;
  hipEventElapsedTime(&ms, ev[2], ev[3]);
  s.accumulate_ms = ms;
  hipEventElapsedTime(&ms, ev[3], ev[4]);
  s.fixup_ms = ms;
  hipEventElapsedTime(&ms, ev[4], ev[5]);
  s.reduce_ms = ms;
  hipEventElapsedTime(&ms, ev[0], ev[5]);
  s.host_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
  s.total_ms = ms + s.host_ms;
  s.window_bits = p.c;
  s.num_windows = p.W;
  s.accumulate_launch_units = p.T;
  s.entries = entries;
  return SV_OK;
}

}  // namespace sv
