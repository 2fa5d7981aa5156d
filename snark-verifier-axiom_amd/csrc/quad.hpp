// XYZZ point arithmetic split over a QUAD of lanes (lane q = lane & 3 holds coordinate q of each
// point: X, Y, ZZ, ZZZ), for the latency-bound tails of the bucket reduction: a full add-2008-s is
// 14 dependent-issue Fq products on one lane (~9 us at one wave per SIMD), here 4 levels of at most
// one product per lane (P, R first, then PP / RR / ZZ1 ZZ2 / ZZZ1 ZZZ2, then PPP / Q / ZZ3, then
// the two halves of Y3 and ZZZ3), the operands of each level exchanged inside the quad by DPP
// quad_perm moves (VALU, no LDS).  Every lane runs the same instruction stream (operand choice by
// v_cndmask), so a product costs one product of latency for the whole quad.  Every perm<>() runs
// unconditionally on all four lanes (never inside a ?: or if whose condition differs across the
// quad: the masked-off source lane would be read as garbage).
//
// 2p domain as xyzz_add_2p (curve.hpp): coordinates in [0, 2p), products lazily reduced, the
// identity exactly ZZ = 0; results are NOT canonical (fe_canon2p before a store that must be).
#pragma once
#include "curve.hpp"

namespace sv {
namespace quad {

constexpr int qp(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }

// every lane of the quad reads lane (CTRL) of its quad (DPP quad_perm)
template <int CTRL>
__device__ __forceinline__ Fq perm(const Fq& a) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[i], CTRL, 0xF, 0xF, false);
  return r;
}
__device__ __forceinline__ Fq pick(bool c, const Fq& a, const Fq& b) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// dbl-2008-s-1 of a: 3 product levels (the identity stays the identity: ZZ3 = V ZZ = 0)
//   1: V = U^2 (U = 2Y) | X^2
//   2: W = U V | S = X V | M^2 (M = 3 X^2) | ZZ3 = V ZZ
//   3: M (S - X3) | W Y | ZZZ3 = W ZZZ ;  X3 = M^2 - 2S, Y3 = M (S - X3) - W Y
__device__ __forceinline__ Fq dbl_2p(const Fq& a, int q) {
  const Fq y = perm<qp(1, 1, 1, 1)>(a), x = perm<qp(0, 0, 0, 0)>(a);
  const Fq u = fe_add2p(y, y);
  const Fq x1 = pick(q == 0, u, x);
  const Fq L1 = fe_mul_lazy(x1, x1);  // q0: V, q1: X^2 (q2, q3: X^2, unused)
  const Fq V = perm<qp(0, 0, 0, 0)>(L1), X2 = perm<qp(1, 1, 1, 1)>(L1);
  const Fq M = fe_add2p(fe_add2p(X2, X2), X2);
  // q0: U V, q1: X V, q2: M M, q3: V ZZ
  const Fq zz = perm<qp(2, 2, 2, 2)>(a);
  const Fq x2 = q == 0 ? u : (q == 1 ? x : (q == 2 ? M : V));
  const Fq y2 = q == 2 ? M : (q == 3 ? zz : V);
  const Fq L2 = fe_mul_lazy(x2, y2);
  const Fq W = perm<qp(0, 0, 0, 0)>(L2), S = perm<qp(1, 1, 1, 1)>(L2), MM = perm<qp(2, 2, 2, 2)>(L2);
  const Fq X3 = fe_sub2p(fe_sub2p(MM, S), S);
  // q0: M (S - X3), q1: W Y, q2: W ZZZ
  const Fq zzz = perm<qp(3, 3, 3, 3)>(a);
  const Fq x3 = q == 0 ? M : W;
  const Fq y3 = q == 0 ? fe_sub2p(S, X3) : (q == 1 ? y : zzz);
  const Fq L3 = fe_mul_lazy(x3, y3);
  const Fq Y3 = fe_sub2p(perm<qp(0, 0, 0, 0)>(L3), perm<qp(1, 1, 1, 1)>(L3));
  const Fq ZZ3 = perm<qp(3, 3, 3, 3)>(L2), ZZZ3 = perm<qp(2, 2, 2, 2)>(L3);
  return q == 0 ? X3 : (q == 1 ? Y3 : (q == 2 ? ZZ3 : ZZZ3));
}

// The rare doubling of an addition (a == b), out of line: one copy in the code instead of one per
// inlined addition (I-cache: an unrolled tree of inlined additions outgrew it)
__device__ __noinline__ Fq dbl_2p_cold(Fq a, int q) { return dbl_2p(a, q); }

// a + b (add-2008-s, complete: identities, a == b, a == -b)
__device__ __forceinline__ Fq add_2p(const Fq& a, const Fq& b, int q) {
  const bool odd = q & 1;
  // level 1: q0 U1 = X1 ZZ2, q1 U2 = X2 ZZ1, q2 S1 = Y1 ZZZ2, q3 S2 = Y2 ZZZ1
  const Fq x1 = pick(odd, perm<qp(0, 0, 1, 1)>(b), perm<qp(0, 0, 1, 1)>(a));
  const Fq y1 = pick(odd, perm<qp(2, 2, 3, 3)>(a), perm<qp(2, 2, 3, 3)>(b));
  const Fq L1 = fe_mul_lazy(x1, y1);
  const Fq pr = perm<qp(1, 0, 3, 2)>(L1);
  const Fq d = fe_sub2p(pick(odd, L1, pr), pick(odd, pr, L1));  // q0, q1: P = U2 - U1; q2, q3: R = S2 - S1
  // level 2: q0 PP = P^2, q1 ZZ1 ZZ2, q2 RR = R^2, q3 ZZZ1 ZZZ2
  const Fq x2 = pick(odd, perm<qp(0, 2, 0, 3)>(a), d);
  const Fq y2 = pick(odd, perm<qp(0, 2, 0, 3)>(b), d);
  const Fq L2 = fe_mul_lazy(x2, y2);
  // level 3: q0 PPP = P PP, q1 Q = U1 PP, q2 ZZ3 = ZZ1 ZZ2 PP (q3 repeats q2)
  const Fq e3 = pick(q == 0, L1, L2);
  const Fq x3 = pick(q == 0, d, perm<qp(0, 0, 1, 1)>(e3));
  const Fq PP = perm<qp(0, 0, 0, 0)>(L2);
  const Fq L3 = fe_mul_lazy(x3, PP);
  const Fq PPP = perm<qp(0, 0, 0, 0)>(L3), Q = perm<qp(1, 1, 1, 1)>(L3);
  const Fq X3 = fe_sub2p(fe_sub2p(fe_sub2p(perm<qp(2, 2, 2, 2)>(L2), PPP), Q), Q);
  // level 4: q0 R (Q - X3), q1 S1 PPP, q2 ZZZ3 = ZZZ1 ZZZ2 PPP (q3 repeats q2)
  const Fq e4 = pick(q == 3, L2, L1);
  const Fq x4 = pick(q == 0, perm<qp(2, 2, 2, 2)>(d), perm<qp(2, 2, 3, 3)>(e4));
  const Fq y4 = pick(q == 0, fe_sub2p(Q, X3), PPP);
  const Fq L4 = fe_mul_lazy(x4, y4);
  const Fq Y3 = fe_sub2p(perm<qp(0, 0, 0, 0)>(L4), perm<qp(1, 1, 1, 1)>(L4));
  const Fq ZZ3 = perm<qp(2, 2, 2, 2)>(L3), ZZZ3 = perm<qp(2, 2, 2, 2)>(L4);
  Fq r = q == 0 ? X3 : (q == 1 ? Y3 : (q == 2 ? ZZ3 : ZZZ3));
  // exceptional cases, per quad (lanes of a quad agree on every flag below)
  const bool a_id = perm<qp(2, 2, 2, 2)>(a).is_zero(), b_id = perm<qp(2, 2, 2, 2)>(b).is_zero();
  const bool p0 = fe_is_zero2p(perm<qp(0, 0, 0, 0)>(d)), r0 = fe_is_zero2p(perm<qp(2, 2, 2, 2)>(d));
  const bool same = !a_id && !b_id && p0 && r0;
  if (__builtin_expect(__any(same), 0)) {  // a == b: double (wave-uniform branch, rare)
    const Fq t = dbl_2p_cold(a, q);
    if (same) r = t;
  }
  if (!a_id && !b_id && p0 && !r0) r = Fq::zero();  // a == -b
  if (b_id) r = a;
  if (a_id) r = b;
  return r;
}

// 4 x 4 transpose inside the quad: lane c holds the four coordinates of ITS point in v[0..3]; after,
// it holds coordinate c of the quad's points 0..3 (two xor rounds of pair swaps)
__device__ __forceinline__ void transpose(Fq v[4], int c) {
  const bool b1 = c & 2, b0 = c & 1;
  {
    const Fq s0 = pick(b1, v[0], v[2]), s1 = pick(b1, v[1], v[3]);
    const Fq r0 = perm<qp(2, 3, 0, 1)>(s0), r1 = perm<qp(2, 3, 0, 1)>(s1);
    v[0] = pick(b1, r0, v[0]);
    v[1] = pick(b1, r1, v[1]);
    v[2] = pick(b1, v[2], r0);
    v[3] = pick(b1, v[3], r1);
  }
  {
    const Fq s0 = pick(b0, v[0], v[1]), s2 = pick(b0, v[2], v[3]);
    const Fq r0 = perm<qp(1, 0, 3, 2)>(s0), r2 = perm<qp(1, 0, 3, 2)>(s2);
    v[0] = pick(b0, r0, v[0]);
    v[1] = pick(b0, v[1], r0);
    v[2] = pick(b0, r2, v[2]);
    v[3] = pick(b0, v[3], r2);
  }
}

// coordinate c (0..3: X, Y, ZZ, ZZZ) of an XYZZ value in memory
__device__ __forceinline__ Fq ld(const G1Xyzz* p, int c) {
  const uint4* q = reinterpret_cast<const uint4*>(p) + 2 * c;
  const uint4 x = q[0], y = q[1];
  Fq r;
  r.v[0] = x.x; r.v[1] = x.y; r.v[2] = x.z; r.v[3] = x.w;
  r.v[4] = y.x; r.v[5] = y.y; r.v[6] = y.z; r.v[7] = y.w;
  return r;
}
__device__ __forceinline__ void st(G1Xyzz* p, int c, const Fq& v) {
  uint4* q = reinterpret_cast<uint4*>(p) + 2 * c;
  q[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  q[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}
// the whole point on every lane of the quad
__device__ __forceinline__ G1Xyzz gather(const Fq& a) {
  return {perm<qp(0, 0, 0, 0)>(a), perm<qp(1, 1, 1, 1)>(a), perm<qp(2, 2, 2, 2)>(a), perm<qp(3, 3, 3, 3)>(a)};
}

// lane + `lanes` (a multiple of 4) of the same coordinate, across the wave
__device__ __forceinline__ Fq down(const Fq& a, int lanes) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)__shfl_down((int)a.v[i], lanes);
  return r;
}

}  // namespace quad
}  // namespace sv
