// KZG decider for BN254 on gfx950: for every accumulator i,
//     e(lhs_i, g2) * e(rhs_i, -s_g2) == 1
// Replaces AccumulationDecider::{decide, decide_all} for KzgAs on NativeLoader
// (snark-verifier/src/pcs/kzg/decider.rs:60-80).
//
// The two G2 points are fixed per call, so their Miller-loop line coefficients (88 steps x 3 Fq2
// each, 33.8 KB for both) are computed once on the host (G2Prepared::from, which the reference
// redoes inside every decide, decider.rs:64) and uploaded.  Each accumulator is then decided by a
// group of 6 x S lanes (below): a 2-term multi-Miller loop with sparse 034 line multiplications and
// the exact final exponentiation (the chain of curve.hpp), Fq12 spread one coefficient per 6 lanes.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

#include "curve.hpp"
#include "decider.hpp"
#include "fq12_lanes.hpp"
#include "runtime.hpp"

namespace sv {

__device__ __forceinline__ G1Aff load_aff_d(const G1Aff* __restrict__ a, uint32_t i, int mont_in) {
  const uint4* p = reinterpret_cast<const uint4*>(a + i);
  uint4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
  G1Aff r;
  r.x.v[0] = q0.x; r.x.v[1] = q0.y; r.x.v[2] = q0.z; r.x.v[3] = q0.w;
  r.x.v[4] = q1.x; r.x.v[5] = q1.y; r.x.v[6] = q1.z; r.x.v[7] = q1.w;
  r.y.v[0] = q2.x; r.y.v[1] = q2.y; r.y.v[2] = q2.z; r.y.v[3] = q2.w;
  r.y.v[4] = q3.x; r.y.v[5] = q3.y; r.y.v[6] = q3.z; r.y.v[7] = q3.w;
  if (!mont_in && !r.is_identity()) {
    r.x = fe_to_mont(r.x);
    r.y = fe_to_mont(r.y);
  }
  return r;
}

// ---------------------------------------------------------------------------------------------
// Lane groups: each accumulator is decided by 6 x S lanes.  Lane (k, s) holds the w^k coefficient
// g_k of the Fq12 accumulator (replicated over its S sub-lanes; fq12_lanes.hpp), and computes the
// products of its coefficient whose index is = s (mod S); the S partial sums are combined with
// cross-lane xor-shuffles, so an Fq12 multiply costs ceil(6/S) Fq2 products of latency, a square
// ceil(4/S), a sparse line step ceil(3/S).  Operands are exchanged through LDS.  Control flow is
// uniform across the wave (identity inputs use the neutral line 1), so the single-wave block can
// use __syncthreads() between the write and read phases of each exchange.
// ---------------------------------------------------------------------------------------------
__constant__ uint32_t c_gamma[3 * 6 * 16] = SV_GAMMA_TAB_INIT;
__constant__ SqrTerm c_sqr[6][4] = SV_SQR_TERMS;
__constant__ int8_t c_naf[ATE_NAF_LEN] = SV_ATE_NAF_INIT;

struct Grp {
  Fq2* a;         // this group's 6 LDS slots for operand A
  Fq2* b;         // ... and operand B
  Fq2* tab;       // kTab x 6 LDS slots: odd powers (and conjugates) for the windowed x-power
  Fq2* keep;      // kKeep x 6 LDS slots: long-lived final-exponentiation values
  int k;          // coefficient index (lanes past 6*S mirror k = 5 and never write)
  int s;          // sub-lane
  bool w;         // writer (s == 0, active)
  SqrTerm sq[4];  // this lane's square terms (slots s, s + S, ...), kept in registers
  SqrTerm sqh;    // S = 8 half-product squaring: term s >> 1 of coefficient k
};

// Cross-lane moves inside 8-lane sub-lane groups by DPP (a VALU operand modifier, no LDS round
// trip like the ds_bpermute behind __shfl_xor): level 1 swaps lane pairs (quad_perm [1,0,3,2]),
// level 2 swaps pairs of pairs (quad_perm [2,3,0,1]); after those every lane of a quad holds the
// quad's sum, so level 3 only needs the other quad of the 8: row_half_mirror (lane i <- 7 - i).
template <int LEVEL>
__device__ __forceinline__ uint32_t dpp_partner(uint32_t x) {
  constexpr int ctrl = LEVEL == 0 ? 0xB1 : (LEVEL == 1 ? 0x4E : 0x141);
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, false);
}

template <int LEVEL>
__device__ __forceinline__ Fq2 dpp_partner(const Fq2& v) {
  Fq2 o;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    o.c0.v[i] = dpp_partner<LEVEL>(v.c0.v[i]);
    o.c1.v[i] = dpp_partner<LEVEL>(v.c1.v[i]);
  }
  return o;
}

template <int S>
__device__ __forceinline__ Fq2 sub_reduce(Fq2 v) {
  // sum over the S consecutive sub-lanes of one coefficient (S = 1, 2, 4, 8; groups 8-aligned)
  static_assert(S == 1 || S == 2 || S == 4 || S == 8, "sub-lane count");
  if constexpr (S >= 2) v = v + dpp_partner<0>(v);
  if constexpr (S >= 4) v = v + dpp_partner<1>(v);
  if constexpr (S >= 8) v = v + dpp_partner<2>(v);
  return v;
}

template <int S>
__device__ __forceinline__ Fq2 g_mul(const Grp& G, const Fq2& x, const Fq2& y) {
  if (G.w) {
    G.a[G.k] = x;
    G.b[G.k] = y;
  }
  __syncthreads();
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int t = 0; t < (6 + S - 1) / S; t++) {
    const int i = t * S + G.s;
    if (i < 6) {
      const int j = G.k - i;
      const Fq2 p = G.a[i] * G.b[j < 0 ? j + 6 : j];
      if (j >= 0) lo = lo + p;
      else hi = hi + p;
    }
  }
  __syncthreads();
  return sub_reduce<S>(lo + fq2_mul_xi(hi));
}

template <int S>
__device__ __forceinline__ Fq2 g_sqr(const Grp& G, const Fq2& x) {
  if (G.w) G.a[G.k] = x;
  __syncthreads();
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int t = 0; t < (4 + S - 1) / S; t++) {
    const int slot = t * S + G.s;
    if (slot < 4) {
      const SqrTerm q = G.sq[t];
      if (q.i >= 0) {
        Fq2 p = G.a[q.i] * G.a[q.j];
        if (q.dbl) p = p + p;
        if (q.xi) hi = hi + p;
        else lo = lo + p;
      }
    }
  }
  __syncthreads();
  return sub_reduce<S>(lo + fq2_mul_xi(hi));
}

// f * (l0 + l1 w + l3 w^3)
template <int S>
__device__ __forceinline__ Fq2 g_line(const Grp& G, const Fq2& x, const Fq2& l0, const Fq2& l1, const Fq2& l3) {
  if (G.w) G.a[G.k] = x;
  __syncthreads();
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int t = 0; t < (3 + S - 1) / S; t++) {
    const int term = t * S + G.s;
    if (term < 3) {
      const int sh = term == 0 ? 0 : (term == 1 ? 1 : 3);
      const int src = G.k - sh;
      const Fq2& l = term == 0 ? l0 : (term == 1 ? l1 : l3);
      const Fq2 p = G.a[src < 0 ? src + 6 : src] * l;
      if (src >= 0) lo = lo + p;
      else hi = hi + p;
    }
  }
  __syncthreads();
  return sub_reduce<S>(lo + fq2_mul_xi(hi));
}

// ---- S = 8 half-product forms: sub-lane s = 2t + h computes component h (0: re, 1: im) of term t
// with two independent Fq products (re(xy) = x0 y0 - x1 y1, im(xy) = x0 y1 + x1 y0) instead of a
// whole Karatsuba Fq2 product (3 dependent-issue products), and its contribution to the
// coefficient: plain (v, 0) / (0, v); wrapped terms carry xi: xi (a + b u) = (9a - b) + (a + 9b) u,
// so a re-lane adds (9v, v) and an im-lane (-v, 9v).  Control flow stays uniform: idle lanes
// compute on slot 0 and contribute zero.
__device__ __forceinline__ Fq fq_mul9(const Fq& a) {
  const Fq a2 = a + a, a4 = a2 + a2;
  return a4 + a4 + a;
}

__device__ __forceinline__ Fq2 half_term(const Fq2& x, const Fq2& y, int h, bool xi, bool live) {
  const Fq m1 = x.c0 * (h ? y.c1 : y.c0);
  const Fq m2 = x.c1 * (h ? y.c0 : y.c1);
  const Fq v = h ? m1 + m2 : fe_sub_lat(m1, m2);
  const Fq v9 = fq_mul9(v);
  Fq cr, ci;
  if (!xi) {
    cr = h ? Fq::zero() : v;
    ci = h ? v : Fq::zero();
  } else {
    cr = h ? -v : v9;
    ci = h ? v9 : v;
  }
  if (!live) cr = ci = Fq::zero();
  return {cr, ci};
}

template <int S>
__device__ __forceinline__ Fq2 g_sqr_h(const Grp& G, const Fq2& x) {
  static_assert(S == 8, "half-product squaring needs 8 sub-lanes");
  if (G.w) G.a[G.k] = x;
  __syncthreads();
  const SqrTerm q = G.sqh;
  const bool live = q.i >= 0;
  const Fq2 X = G.a[live ? q.i : 0], Y = G.a[live ? q.j : 0];
  Fq2 c = half_term(X, Y, G.s & 1, q.xi, live);
  if (q.dbl) c = c + c;
  __syncthreads();
  return sub_reduce<S>(c);
}

// f * (l0 + l1 w + l3 w^3): terms t = 0, 1, 2 take f_k, f_{k-1}, f_{k-3} (wrapping with xi)
template <int S>
__device__ __forceinline__ Fq2 g_line_h(const Grp& G, const Fq2& x, const Fq2& l0, const Fq2& l1, const Fq2& l3) {
  static_assert(S == 8, "half-product line step needs 8 sub-lanes");
  if (G.w) G.a[G.k] = x;
  __syncthreads();
  const int t = G.s >> 1;
  const bool live = t < 3;
  const int sh = t == 0 ? 0 : (t == 1 ? 1 : 3);
  const int src = G.k - sh;
  const Fq2& l = t == 0 ? l0 : (t == 1 ? l1 : l3);
  const Fq2 c = half_term(G.a[live ? (src < 0 ? src + 6 : src) : 0], l, G.s & 1, src < 0, live);
  __syncthreads();
  return sub_reduce<S>(c);
}

__device__ __forceinline__ Fq2 g_conj(const Grp& G, const Fq2& x) { return (G.k & 1) ? -x : x; }
__device__ __forceinline__ Fq2 g_frob(const Grp& G, int n, const Fq2& x) {
  Fq2 y = (n & 1) ? fq2_conj(x) : x;
  if (G.k == 0) return y;
  const uint32_t* t = c_gamma + ((n - 1) * 6 + G.k) * 16;
  Fq2 c;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c.c0.v[i] = t[i];
    c.c1.v[i] = t[8 + i];
  }
  return y * c;
}
// f^-1 = conj(f) N^-1 with N = f conj(f) = a^2 - v b^2 in Fq6 (f = a + b w over Fq6, v = w^2):
// N sits on the even w-coefficients, its Fq6 inverse (t0 + t1 v + t2 v^2) / d is formed with the
// three t_j on the lanes of coefficients 0, 2, 4 in parallel, and only the norm of d in Fq is
// inverted (one fe_inv, on every lane, uniform) -- instead of a whole Fq12 inversion per lane.
template <int S>
__device__ __forceinline__ Fq2 g_inv(const Grp& G, const Fq2& f) {
  const Fq2 fc = g_conj(G, f);
  const Fq2 nk = g_mul<S>(G, f, fc);  // odd coefficients vanish
  if (G.w) G.a[G.k] = nk;
  __syncthreads();
  const Fq2 c0 = G.a[0], c1 = G.a[2], c2 = G.a[4];
  const int j = G.k >> 1;
  // t0 = c0^2 - xi c1 c2, t1 = xi c2^2 - c0 c1, t2 = c1^2 - c0 c2 (lanes of coefficient 2j)
  const Fq2 x = j == 0 ? c0 : (j == 1 ? c2 : c1);
  const Fq2 y0 = j == 0 ? c1 : c0, y1 = j == 0 ? c2 : (j == 1 ? c1 : c2);
  const Fq2 sq = x * x, pr = y0 * y1;
  const Fq2 tj = j == 0 ? sq - fq2_mul_xi(pr) : (j == 1 ? fq2_mul_xi(sq) - pr : sq - pr);
  __syncthreads();
  if (G.w && !(G.k & 1)) G.b[j] = tj;
  __syncthreads();
  const Fq2 t0 = G.b[0], t1 = G.b[1], t2 = G.b[2];
  __syncthreads();
  const Fq2 d = c0 * t0 + fq2_mul_xi(c2 * t1 + c1 * t2);
  const Fq2 di = fq2_inv(d);
  const Fq2 ninv = (G.k & 1) ? Fq2::zero() : (j == 0 ? t0 : (j == 1 ? t1 : t2)) * di;
  return g_mul<S>(G, fc, ninv);
}
// Squaring / line steps: the half-product forms at S = 8, the whole-product forms otherwise
// (measured per op on one wave, tools/ubench_decops.hip: g_sqr 4.8 us, g_sqr_h 3.2 us; a Granger-Scott
// cyclotomic squaring with one product level measured 6.1 us -- single-wave code is bound by
// dependent-instruction latency, and its many Fq2 additions cost more than the products it saves)
template <int S>
__device__ __forceinline__ Fq2 g_msq(const Grp& G, const Fq2& x) {
  if constexpr (S == 8) return g_sqr_h<S>(G, x);
  else return g_sqr<S>(G, x);
}
template <int S>
__device__ __forceinline__ Fq2 g_mline(const Grp& G, const Fq2& x, const Fq2& l0, const Fq2& l1, const Fq2& l3) {
  if constexpr (S == 8) return g_line_h<S>(G, x, l0, l1, l3);
  else return g_line<S>(G, x, l0, l1, l3);
}

// f * y with y's six coefficients already in LDS (yb[0..5]): no operand write on the critical path
template <int S>
__device__ __forceinline__ Fq2 g_mul_lds(const Grp& G, const Fq2& x, const Fq2* yb) {
  if (G.w) G.a[G.k] = x;
  __syncthreads();
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int t = 0; t < (6 + S - 1) / S; t++) {
    const int i = t * S + G.s;
    if (i < 6) {
      const int j = G.k - i;
      const Fq2 p = G.a[i] * yb[j < 0 ? j + 6 : j];
      if (j >= 0) lo = lo + p;
      else hi = hi + p;
    }
  }
  __syncthreads();
  return sub_reduce<S>(lo + fq2_mul_xi(hi));
}

__device__ __forceinline__ void g_put(const Grp& G, Fq2* slots, int e, const Fq2& v) {
  if (G.w) slots[e * 6 + G.k] = v;
}
__device__ __forceinline__ Fq2 g_get(const Grp& G, const Fq2* slots, int e) { return slots[e * 6 + G.k]; }

// x = 0x44e992b44a6909f1 in width-4 NAF (odd digits in [-7, 7], 14 non-zero of 63): 62 squarings
// and 13 multiplications by a tabulated odd power instead of 27 for plain binary.  Negative digits
// multiply by the conjugate, which is the inverse on the cyclotomic subgroup the hard part of the
// final exponentiation works in.
struct XNaf {
  int8_t d[66];
  int len;
};
constexpr XNaf make_xnaf() {
  XNaf r{};
  uint64_t k = BN_X;
  int i = 0;
  while (k) {
    int v = 0;
    if (k & 1) {
      v = (int)(k & 15);
      if (v >= 8) v -= 16;
      k = v >= 0 ? k - (uint64_t)v : k + (uint64_t)(-v);
    }
    r.d[i++] = (int8_t)v;
    k >>= 1;
  }
  r.len = i;
  return r;
}
__constant__ XNaf c_xnaf = make_xnaf();
static constexpr int kTab = 8;   // a, a^3, a^5, a^7, then their conjugates
static constexpr int kKeep = 6;

template <int S>
__device__ __forceinline__ Fq2 g_pow_x(const Grp& G, const Fq2& a) {
  const Fq2 a2 = g_msq<S>(G, a);
  g_put(G, G.tab, 0, a);
  g_put(G, G.tab, 4, g_conj(G, a));
  Fq2 ak = a;
  for (int e = 1; e < 4; e++) {
    ak = g_mul<S>(G, ak, a2);
    g_put(G, G.tab, e, ak);
    g_put(G, G.tab, 4 + e, g_conj(G, ak));
  }
  __syncthreads();  // the last table entries are read below without an intervening exchange
  const int len = c_xnaf.len;
  const int top = c_xnaf.d[len - 1];
  Fq2 r = g_get(G, G.tab, top > 0 ? (top - 1) / 2 : 4 + (-top - 1) / 2);
  for (int i = len - 2; i >= 0; i--) {
    r = g_msq<S>(G, r);
    const int d = c_xnaf.d[i];
    if (d) r = g_mul_lds<S>(G, r, G.tab + 6 * (d > 0 ? (d - 1) / 2 : 4 + (-d - 1) / 2));
  }
  return r;
}

// Prologue: the group's lanes evaluate all 2 x ATE_NUM_LINES lines at their accumulator's points
// into LDS (l0 = c0 yP, l1 = c3 xP, l3 = c4; the neutral line 1 when P is the identity), so the
// Miller loop's line steps do no global loads and no line arithmetic on the critical path.
__device__ __forceinline__ void eval_lines(LineCoeff* __restrict__ E, const LineCoeff* __restrict__ L1,
                                           const LineCoeff* __restrict__ L2, const G1Aff& p1, const G1Aff& p2,
                                           int lane_in_group, int group_lanes) {
  for (int it = lane_in_group; it < 2 * ATE_NUM_LINES; it += group_lanes) {
    const int idx = it >> 1;
    const bool second = it & 1;
    const G1Aff& p = second ? p2 : p1;
    LineCoeff out;
    if (!p.is_identity()) {
      const LineCoeff c = (second ? L2 : L1)[idx];
      out.c0 = c.c0 * p.y;
      out.c3 = c.c3 * p.x;
      out.c4 = c.c4;
    } else {
      out.c0 = Fq2::one();
      out.c3 = Fq2::zero();
      out.c4 = Fq2::zero();
    }
    E[it] = out;
  }
}

// ---- Step multipliers (S = 8 path): the Miller loop's line products are known once the lines are
// evaluated, so the prologue folds them off the critical path.  Pair idx (the lines of both G2
// points at one step) becomes the 5-sparse D_idx = (a0 + a1 w + a3 w^3)(b0 + b1 w + b3 w^3), and a
// step with an addition (or the final Frobenius steps) multiplies its two pairs into a dense M.
// The loop then costs one square and ONE multiplication per step (66) instead of a square and
// 2-4 sparse line steps (176).
struct MergeTab {
  int8_t first[32];  // first pair index of each merged step (the second is first + 1)
  int n;
};
constexpr MergeTab make_merges() {
  MergeTab t{};
  int idx = 0, m = 0;
  for (int i = ATE_NAF_LEN - 1; i >= 1; i--) {
    if (ATE_NAF[i - 1] != 0) {
      t.first[m++] = (int8_t)idx;
      idx += 2;
    } else {
      idx += 1;
    }
  }
  t.first[m++] = (int8_t)idx;  // the two Frobenius steps
  t.n = m;
  return t;
}
__constant__ MergeTab c_merge = make_merges();
static constexpr int kMaxMerge = 32;

// D_idx for pairs idx = lane, lane + lanes, ...: 6 Fq2 products (Karatsuba on the three cross terms)
__device__ __forceinline__ void pair_products(Fq2* __restrict__ D, const LineCoeff* __restrict__ E, int lane,
                                              int lanes) {
  for (int idx = lane; idx < ATE_NUM_LINES; idx += lanes) {
    const LineCoeff A = E[2 * idx], Bq = E[2 * idx + 1];
    const Fq2 m00 = A.c0 * Bq.c0, m11 = A.c3 * Bq.c3, m33 = A.c4 * Bq.c4;
    const Fq2 x01 = (A.c0 + A.c3) * (Bq.c0 + Bq.c3);
    const Fq2 x03 = (A.c0 + A.c4) * (Bq.c0 + Bq.c4);
    const Fq2 x13 = (A.c3 + A.c4) * (Bq.c3 + Bq.c4);
    Fq2* d = D + 6 * idx;
    d[0] = m00 + fq2_mul_xi(m33);
    d[1] = x01 - m00 - m11;
    d[2] = m11;
    d[3] = x03 - m00 - m33;
    d[4] = x13 - m11 - m33;
    d[5] = Fq2::zero();
  }
}

// M_m = D_a D_{a+1} (both 5-sparse) for every merged step; job = (step, output coefficient)
__device__ __forceinline__ void merge_products(Fq2* __restrict__ M, const Fq2* __restrict__ D, int lane, int lanes) {
  for (int job = lane; job < c_merge.n * 6; job += lanes) {
    const int m = job / 6, k = job % 6;
    const Fq2* a = D + 6 * c_merge.first[m];
    const Fq2* b = a + 6;
    Fq2 lo = Fq2::zero(), hi = Fq2::zero();
    for (int i = 0; i < 5; i++) {
      const int j = k - i;
      if (j >= 0 && j < 5) lo = lo + a[i] * b[j];
      const int jw = k + 6 - i;
      if (jw >= 0 && jw < 5) hi = hi + a[i] * b[jw];
    }
    M[6 * m + k] = lo + fq2_mul_xi(hi);
  }
}

template <int S>
__global__ void __launch_bounds__(64) k_decide_lanes(const G1Aff* __restrict__ lhs, const G1Aff* __restrict__ rhs,
                                                      uint32_t n, const LineCoeff* __restrict__ L1,
                                                      const LineCoeff* __restrict__ L2, int mont_in,
                                                      int32_t* __restrict__ verdict, Fq12* __restrict__ gt,
                                                      int phases) {
  constexpr int GL = 8 * S;         // lanes per group (6 * S active)
  constexpr int NGRP = 64 / GL;     // groups per single-wave block
  __shared__ Fq2 sh[2 * NGRP * 6];
  __shared__ LineCoeff ev[NGRP][2 * ATE_NUM_LINES];
  __shared__ Fq2 tabk[NGRP][(kTab + kKeep) * 6];
  constexpr bool kMerged = S == 8;  // one group per wave: room for the step multipliers in LDS
  __shared__ Fq2 dmul[kMerged ? ATE_NUM_LINES * 6 : 1];
  const int lane = threadIdx.x, grp = lane / GL, gl = lane % GL;
  const bool active = gl < 6 * S;
  const int k = active ? gl / S : 5, sub = active ? gl % S : 0;
  const uint32_t acc = blockIdx.x * NGRP + grp;
  Grp G{sh + grp * 12, sh + grp * 12 + 6, tabk[grp], tabk[grp] + kTab * 6, k, sub, active && sub == 0, {}, {}};
  G.sqh = (S == 8 && active) ? c_sqr[k][sub >> 1] : SqrTerm{-1, -1, 0, 0};
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int slot = t * S + sub;
    G.sq[t] = slot < 4 ? c_sqr[k][slot] : SqrTerm{-1, -1, 0, 0};
  }
  const bool valid = acc < n;
  G1Aff p1 = {Fq::zero(), Fq::zero()}, p2 = p1;
  if (valid) {
    p1 = load_aff_d(lhs, acc, mont_in);
    p2 = load_aff_d(rhs, acc, mont_in);
  }
  eval_lines(ev[grp], L1, L2, p1, p2, gl, GL);
  __syncthreads();
  const LineCoeff* E = ev[grp];
  Fq2 f = G.k == 0 ? Fq2::one() : Fq2::zero();
  int idx = 0;
  if constexpr (kMerged) {
    pair_products(dmul, E, gl, GL);
    __syncthreads();
    Fq2* M = reinterpret_cast<Fq2*>(ev[grp]);  // the evaluated lines are dead now
    static_assert(sizeof(ev[0]) >= kMaxMerge * 6 * sizeof(Fq2), "merged steps must fit the line buffer");
    merge_products(M, dmul, gl, GL);
    __syncthreads();
    int m = 0;
    for (int i = ATE_NAF_LEN - 1; i >= 1 && (phases & 1); i--) {
      const Fq2* mul = c_naf[i - 1] != 0 ? M + 6 * m++ : dmul + 6 * idx;
      idx += c_naf[i - 1] != 0 ? 2 : 1;
      if (i == ATE_NAF_LEN - 1) f = mul[G.k];  // f = 1 * mul
      else f = g_mul_lds<S>(G, g_msq<S>(G, f), mul);
    }
    if (phases & 1) f = g_mul_lds<S>(G, f, M + 6 * m);  // the two Frobenius steps
  } else {
    for (int i = ATE_NAF_LEN - 1; i >= 1 && (phases & 1); i--) {
      if (i != ATE_NAF_LEN - 1) f = g_msq<S>(G, f);
      f = g_mline<S>(G, f, E[2 * idx].c0, E[2 * idx].c3, E[2 * idx].c4);
      f = g_mline<S>(G, f, E[2 * idx + 1].c0, E[2 * idx + 1].c3, E[2 * idx + 1].c4);
      idx++;
      if (c_naf[i - 1] != 0) {
        f = g_mline<S>(G, f, E[2 * idx].c0, E[2 * idx].c3, E[2 * idx].c4);
        f = g_mline<S>(G, f, E[2 * idx + 1].c0, E[2 * idx + 1].c3, E[2 * idx + 1].c4);
        idx++;
      }
    }
    for (int st = 0; st < 2 && (phases & 1); st++) {
      f = g_mline<S>(G, f, E[2 * idx].c0, E[2 * idx].c3, E[2 * idx].c4);
      f = g_mline<S>(G, f, E[2 * idx + 1].c0, E[2 * idx + 1].c3, E[2 * idx + 1].c4);
      idx++;
    }
  }
  // final exponentiation (same chain as curve.hpp final_exponentiation)
  // (phases: debug/profiling knob SVGPU_DECIDER_PHASES, 3 = both halves; results are only valid at 3)
  Fq2 e = f;
  if (phases & 2) {
  Fq2 fi = g_inv<S>(G, f);
  f = g_mul<S>(G, g_conj(G, f), fi);
  f = g_mul<S>(G, g_frob(G, 2, f), f);
  // hard part: f^(l0 + l1 p + l2 p^2 + p^3) with the x-power chain; the small powers of fx and
  // fx^2 share their ladders (fx^6 -> fx^12 -> fx^18, fx2^6 -> fx2^12 -> fx2^18 -> fx2^30)
  enum { K_F, K_B12, K_B18, K_A6, K_A18, K_A30 };
  g_put(G, G.keep, K_F, f);
  const Fq2 fx = g_pow_x<S>(G, f);
  {
    const Fq2 b6 = g_msq<S>(G, g_mul<S>(G, g_msq<S>(G, fx), fx));
    const Fq2 b12 = g_msq<S>(G, b6);
    g_put(G, G.keep, K_B12, b12);
    g_put(G, G.keep, K_B18, g_mul<S>(G, b12, b6));
  }
  const Fq2 fx2 = g_pow_x<S>(G, fx);
  {
    const Fq2 a6 = g_msq<S>(G, g_mul<S>(G, g_msq<S>(G, fx2), fx2));
    const Fq2 a12 = g_msq<S>(G, a6);
    const Fq2 a18 = g_mul<S>(G, a12, a6);
    g_put(G, G.keep, K_A6, a6);
    g_put(G, G.keep, K_A18, a18);
    g_put(G, G.keep, K_A30, g_mul<S>(G, a18, a12));
  }
  const Fq2 fx3 = g_pow_x<S>(G, fx2);
  Fq2 y = g_msq<S>(G, g_msq<S>(G, g_msq<S>(G, fx3)));        // fx3^8
  const Fq2 y36 = g_msq<S>(G, g_msq<S>(G, g_mul<S>(G, y, fx3)));  // fx3^36
  f = g_get(G, G.keep, K_F);
  const Fq2 l2v = g_mul_lds<S>(G, f, G.keep + 6 * K_A6);
  Fq2 t = g_mul_lds<S>(G, g_mul_lds<S>(G, y36, G.keep + 6 * K_A18), G.keep + 6 * K_B12);
  const Fq2 l1v = g_mul_lds<S>(G, g_conj(G, t), G.keep + 6 * K_F);
  t = g_mul_lds<S>(G, g_mul_lds<S>(G, y36, G.keep + 6 * K_A30), G.keep + 6 * K_B18);
  t = g_mul<S>(G, t, g_msq<S>(G, f));
  const Fq2 l0v = g_conj(G, t);
  e = g_mul<S>(G, g_mul<S>(G, g_mul<S>(G, l0v, g_frob(G, 1, l1v)), g_frob(G, 2, l2v)), g_frob(G, 3, f));
  }
  const bool one_k = G.k == 0 ? (e == Fq2::one()) : e.is_zero();
  const uint64_t bal = __ballot(one_k || !active);
  const uint64_t gmask = GL == 64 ? ~0ull : ((1ull << GL) - 1);
  const bool ok = ((bal >> (grp * GL)) & gmask) == gmask;
  if (valid && G.w) {
    if (G.k == 0) verdict[acc] = ok ? 1 : 0;
    if (gt) {
      Fq2* dst = reinterpret_cast<Fq2*>(gt + acc) + (G.k & 1) * 3 + (G.k >> 1);
      *dst = e;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Host side: prepared-line cache.  Each deciding key's lines live in their own immutable device
// buffer, shared by refcount: a call holds its entry until its stream has synchronised, so a
// concurrent call with another key (a second verifier on another rayon worker) uploads into a NEW
// buffer and can never overwrite lines a running kernel reads.  A few keys are kept per device
// (verifiers rarely switch keys); an evicted entry is freed when its last in-flight call drops it.
// ---------------------------------------------------------------------------------------------
namespace {
struct LineEntry {
  unsigned char key[2 * sizeof(G2Aff)];
  int device = 0;
  LineCoeff* d_lines = nullptr;  // 2 * ATE_NUM_LINES, written once before the entry is published
  ~LineEntry() {
    if (d_lines) {
      int prev = 0;
      (void)hipGetDevice(&prev);
      (void)hipSetDevice(device);
      (void)hipFree(d_lines);
      (void)hipSetDevice(prev);
    }
  }
};
constexpr int kLineCacheKeys = 4;
struct LineCache {
  std::mutex mu;
  std::shared_ptr<LineEntry> e[kLineCacheKeys];  // most recently used first
};
// leaked on purpose: cached entries must not hipFree from static destructors after HIP teardown
LineCache* const g_cache = new LineCache[64];
}  // namespace

static G2Aff g2_from_abi(const sv_g2_affine* q, int mont_in) {
  G2Aff r;
  memcpy(&r.x.c0, &q->x.c0, 32);
  memcpy(&r.x.c1, &q->x.c1, 32);
  memcpy(&r.y.c0, &q->y.c0, 32);
  memcpy(&r.y.c1, &q->y.c1, 32);
  if (!mont_in) {
    r.x.c0 = fe_to_mont(r.x.c0);
    r.x.c1 = fe_to_mont(r.x.c1);
    r.y.c0 = fe_to_mont(r.y.c0);
    r.y.c1 = fe_to_mont(r.y.c1);
  }
  return r;
}

static bool g2_on_twist(const G2Aff& q) {
  Fq2 lhs = fq2_sqr(q.y);
  Fq2 rhs = fq2_sqr(q.x) * q.x + fq2_const(TWIST_B_C0, TWIST_B_C1);
  return lhs == rhs;
}

// The caller keeps `*out` alive until every kernel reading its lines has finished.
static int decider_lines(const sv_g2_affine* g2, const sv_g2_affine* s_g2, int form, int device,
                         hipStream_t st, std::shared_ptr<LineEntry>* out) {
  if (device < 0 || device >= 64) return SV_ERR_ARG;
  G2Aff q1 = g2_from_abi(g2, form == SV_MONTGOMERY);
  G2Aff q2 = g2_from_abi(s_g2, form == SV_MONTGOMERY);
  if (q1.is_identity() || q2.is_identity() || !g2_on_twist(q1) || !g2_on_twist(q2)) {
    set_error("deciding key G2 point is the identity or not on the twist");
    return SV_ERR_ARG;
  }
  q2.y = -q2.y;  // -s_g2
  unsigned char key[sizeof(LineEntry::key)];
  memcpy(key, &q1, sizeof(G2Aff));
  memcpy(key + sizeof(G2Aff), &q2, sizeof(G2Aff));
  LineCache& c = g_cache[device];
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (int i = 0; i < kLineCacheKeys; i++) {
      if (c.e[i] && memcmp(key, c.e[i]->key, sizeof key) == 0) {
        std::shared_ptr<LineEntry> hit = c.e[i];
        for (int j = i; j > 0; j--) c.e[j] = c.e[j - 1];
        c.e[0] = hit;
        *out = std::move(hit);
        return SV_OK;
      }
    }
  }
  // miss: prepare and upload outside the lock into a fresh buffer, then publish
  auto ent = std::make_shared<LineEntry>();
  memcpy(ent->key, key, sizeof key);
  ent->device = device;
  std::vector<LineCoeff> h(2 * ATE_NUM_LINES);
  g2_prepare(q1, h.data());
  g2_prepare(q2, h.data() + ATE_NUM_LINES);
  SV_HIP(hipMalloc(&ent->d_lines, h.size() * sizeof(LineCoeff)));
  SV_HIP(hipMemcpyAsync(ent->d_lines, h.data(), h.size() * sizeof(LineCoeff), hipMemcpyHostToDevice, st));
  SV_HIP(hipStreamSynchronize(st));
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (int j = kLineCacheKeys - 1; j > 0; j--) c.e[j] = c.e[j - 1];
    c.e[0] = ent;
  }
  *out = std::move(ent);
  return SV_OK;
}

int decide_run_device(const sv_g2_affine* g2, const sv_g2_affine* s_g2, const void* d_lhs,
                      const void* d_rhs, size_t n, int form, int device, hipStream_t user_stream,
                      int32_t* first_fail, int32_t* verdicts_host, sv_fq12* gt_host) {
  if (n == 0) {
    set_error("accumulators should not be empty");
    return SV_ERR_EMPTY;
  }
  if (form != SV_CANONICAL && form != SV_MONTGOMERY) {
    set_error("bad form %d", form);
    return SV_ERR_ARG;
  }
  WsLease lease(device, user_stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  hipStream_t st = ws->stream;
  std::shared_ptr<LineEntry> line_ref;  // held until the stream has synchronised (below)
  SV_TRY(decider_lines(g2, s_g2, form, device, st, &line_ref));
  const LineCoeff* lines = line_ref->d_lines;
  size_t bytes = Workspace::aligned(n * 4) + (gt_host ? Workspace::aligned(n * sizeof(Fq12)) : 0);
  SV_TRY(ws->reserve(bytes));
  SV_TRY(ws->reserve_pinned(n * 4 + 256));
  int32_t* d_verdict = ws->carve<int32_t>(n);
  Fq12* d_gt = gt_host ? ws->carve<Fq12>(n) : nullptr;
  SV_HIP(hipEventRecord(ws->ev[0], st));
  // SVGPU_DECIDER_LANES = 48 (6 x 8 lanes per accumulator, 1 per wave; default) or 24 (6 x 4, 2 per wave)
  static const int lanes = getenv("SVGPU_DECIDER_LANES") ? atoi(getenv("SVGPU_DECIDER_LANES")) : 48;
  static const int phases = getenv("SVGPU_DECIDER_PHASES") ? atoi(getenv("SVGPU_DECIDER_PHASES")) : 3;
  const G1Aff* dl = reinterpret_cast<const G1Aff*>(d_lhs);
  const G1Aff* dr = reinterpret_cast<const G1Aff*>(d_rhs);
  const int mont = form == SV_MONTGOMERY ? 1 : 0;
  const LineCoeff* L2 = lines + ATE_NUM_LINES;
  if (lanes == 48)
    hipLaunchKernelGGL(k_decide_lanes<8>, dim3((unsigned)n), dim3(64), 0, st, dl, dr, (uint32_t)n, lines, L2, mont,
                       d_verdict, d_gt, phases);
  else
    hipLaunchKernelGGL(k_decide_lanes<4>, dim3((unsigned)((n + 1) / 2)), dim3(64), 0, st, dl, dr, (uint32_t)n,
                       lines, L2, mont, d_verdict, d_gt, phases);
  SV_HIP(hipGetLastError());
  SV_HIP(hipEventRecord(ws->ev[1], st));
  int32_t* hv = reinterpret_cast<int32_t*>(ws->pinned);
  SV_HIP(hipMemcpyAsync(hv, d_verdict, n * 4, hipMemcpyDeviceToHost, st));
  if (gt_host) {
    std::vector<Fq12> tmp(n);
    SV_HIP(hipMemcpyAsync(tmp.data(), d_gt, n * sizeof(Fq12), hipMemcpyDeviceToHost, st));
    SV_HIP(hipStreamSynchronize(st));
    for (size_t i = 0; i < n; i++) {
      const Fq2* c[6] = {&tmp[i].c0.c0, &tmp[i].c0.c1, &tmp[i].c0.c2,
                         &tmp[i].c1.c0, &tmp[i].c1.c1, &tmp[i].c1.c2};
      for (int k = 0; k < 6; k++) {
        Fq a = fe_from_mont(c[k]->c0), b = fe_from_mont(c[k]->c1);
        memcpy(&gt_host[i].c[k].c0, a.v, 32);
        memcpy(&gt_host[i].c[k].c1, b.v, 32);
      }
    }
  }
  SV_HIP(hipStreamSynchronize(st));
  float ms = 0;
  hipEventElapsedTime(&ms, ws->ev[0], ws->ev[1]);
  decider_last_kernel_ms() = ms;
  int32_t ff = -1;
  for (size_t i = 0; i < n; i++) {
    if (verdicts_host) verdicts_host[i] = hv[i];
    if (ff < 0 && !hv[i]) ff = (int32_t)i;
  }
  if (first_fail) *first_fail = ff;
  return SV_OK;
}

float& decider_last_kernel_ms() {
  static thread_local float v = 0;
  return v;
}

}  // namespace sv
