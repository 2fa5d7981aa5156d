// BN254 G1 (y^2 = x^3 + 3) in XYZZ coordinates, plus the optimal-ate pairing pieces.
//
// XYZZ (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2; identity ZZ = 0) is the bucket representation of the
// Pippenger kernels: a mixed add (bucket += affine) is 8M + 2S, a full add 12M + 2S.  Formulas:
// EFD "g1p/auto-shortw-xyzz" madd-2008-s, add-2008-s, dbl-2008-s-1, mdbl-2008-s-1, with the
// exceptional cases (P == Q, P == -Q, identities) handled explicitly, because the reference's
// halo2curves group law is complete and MSM inputs may repeat bases or contain P and -P.
//
// Pairing: D-type twist, homogeneous-projective G2 line coefficients (c0, c3, c4) evaluated at
// P as (c0 * yP, c3 * xP, c4) and folded in with the sparse 034 multiplication; final
// exponentiation is the EXACT (p^12-1)/r power (easy part, then the hard part via its p-adic
// digits in x), so Gt values match oracle/bn254.py's direct exponentiation bit for bit.
#pragma once
#include "field.hpp"

namespace sv {

struct G1Aff {  // Montgomery coordinates; identity encoded (0, 0) as in halo2curves
  Fq x, y;
  SV_HD bool is_identity() const { return x.is_zero() && y.is_zero(); }
};

struct G1Xyzz {
  Fq X, Y, ZZ, ZZZ;
  SV_HD static G1Xyzz identity() { return {Fq::zero(), Fq::zero(), Fq::zero(), Fq::zero()}; }
  SV_HD bool is_identity() const { return ZZ.is_zero(); }
  SV_HD static G1Xyzz from_affine(const G1Aff& p) {
    if (p.is_identity()) return identity();
    return {p.x, p.y, Fq::one(), Fq::one()};
  }
};

// a b - c d with one Montgomery reduction (fe_mul_sum over (a, c) x (b, -d)): the Y3 of every
// XYZZ formula, 192 instead of 256 multiply-adds.
SV_HD Fq mul_diff(const Fq& a, const Fq& b, const Fq& c, const Fq& d) {
  const Fq x[2] = {a, c};
  const Fq y[2] = {b, -d};
  return fe_mul_sum(x, y);
}

// dbl-2008-s-1 (a = 0)
SV_HD G1Xyzz xyzz_dbl(const G1Xyzz& p) {
  if (p.is_identity()) return p;
  Fq U = fe_dbl(p.Y);
  Fq V = fe_sqr_hp(U);
  Fq W = U * V;
  Fq S = p.X * V;
  Fq X2 = fe_sqr_hp(p.X);
  Fq M = fe_dbl(X2) + X2;
  Fq X3 = fe_sqr_hp(M) - fe_dbl(S);
  Fq Y3 = mul_diff(M, S - X3, W, p.Y);
  return {X3, Y3, V * p.ZZ, W * p.ZZZ};
}

// mdbl-2008-s-1: double an affine point (not identity)
SV_HD G1Xyzz xyzz_mdbl(const Fq& x, const Fq& y) {
  Fq U = fe_dbl(y);
  Fq V = fe_sqr_hp(U);
  Fq W = U * V;
  Fq S = x * V;
  Fq X2 = fe_sqr_hp(x);
  Fq M = fe_dbl(X2) + X2;
  Fq X3 = fe_sqr_hp(M) - fe_dbl(S);
  Fq Y3 = mul_diff(M, S - X3, W, y);
  return {X3, Y3, V, W};
}

// madd-2008-s: p (XYZZ) + (x2, y2) affine, (x2, y2) not identity.
SV_HD G1Xyzz xyzz_madd(const G1Xyzz& p, const Fq& x2, const Fq& y2) {
  if (p.is_identity()) return {x2, y2, Fq::one(), Fq::one()};
  Fq U2 = x2 * p.ZZ;
  Fq S2 = y2 * p.ZZZ;
  Fq Pd = U2 - p.X;
  Fq Rd = S2 - p.Y;
  if (Pd.is_zero()) {
    if (Rd.is_zero()) return xyzz_mdbl(x2, y2);
    return G1Xyzz::identity();
  }
  Fq PP = fe_sqr_hp(Pd);
  Fq PPP = Pd * PP;
  Fq Q = p.X * PP;
  Fq X3 = fe_sqr_hp(Rd) - PPP - fe_dbl(Q);
  Fq Y3 = mul_diff(Rd, Q - X3, p.Y, PPP);
  return {X3, Y3, p.ZZ * PP, p.ZZZ * PPP};
}

SV_HD G1Xyzz xyzz_madd_aff(const G1Xyzz& p, const G1Aff& q) {
  if (q.is_identity()) return p;
  return xyzz_madd(p, q.x, q.y);
}

// madd-2008-s with the accumulator kept in the 2p domain (coordinates in [0, 2p), field.hpp): the
// products skip their final conditional subtraction, 2Q is subtracted as Q twice, and the
// degenerate-case tests compare against both representatives of 0.  Y3 = Rd (Q - X3) - Y PPP is
// one fused sum of two products of inputs below 2p: below 2.52 p before, 1.52 p after its
// subtraction.  For the bucket accumulation chain (k_accumulate), which canonicalises before every
// store (xyzz_canon2p); (x2, y2) is a reduced affine point, not the identity.
SV_HD G1Xyzz xyzz_madd_2p(const G1Xyzz& p, const Fq& x2, const Fq& y2) {
  if (p.is_identity()) return {x2, y2, Fq::one(), Fq::one()};
  const Fq U2 = fe_mul_lazy(x2, p.ZZ);
  const Fq S2 = fe_mul_lazy(y2, p.ZZZ);
  const Fq Pd = fe_sub2p(U2, p.X);
  const Fq Rd = fe_sub2p(S2, p.Y);
  if (fe_is_zero2p(Pd)) {
    if (fe_is_zero2p(Rd)) return xyzz_mdbl(x2, y2);
    return G1Xyzz::identity();
  }
  const Fq PP = fe_sqr_hp<FqTag, false>(Pd);
  const Fq PPP = fe_mul_lazy(Pd, PP);
  const Fq Q = fe_mul_lazy(p.X, PP);
  const Fq X3 = fe_sub2p(fe_sub2p(fe_sub2p(fe_sqr_hp<FqTag, false>(Rd), PPP), Q), Q);
  const Fq x[2] = {Rd, p.Y};
  const Fq y[2] = {fe_sub2p(Q, X3), fe_neg2p(PPP)};
  return {X3, fe_mul_sum(x, y), fe_mul_lazy(p.ZZ, PP), fe_mul_lazy(p.ZZZ, PPP)};
}
// xyzz_madd_2p with the doubling case (p = (x2, y2)) run through the addition's own products, as
// r29::madd (curve29.hpp): mdbl's U = 2 y2, M = 3 x2^2 become Pd and Rd, (X, Y, ZZ, ZZZ) =
// (x2, y2, 1, 1), and X3 drops its PPP term -- the rare branch only sets operands.
SV_HD G1Xyzz xyzz_madd_2p_u(const G1Xyzz& p, const Fq& x2, const Fq& y2) {
  if (p.is_identity()) return {x2, y2, Fq::one(), Fq::one()};
  Fq Pd = fe_sub2p(fe_mul_lazy(x2, p.ZZ), p.X);
  Fq Rd = fe_sub2p(fe_mul_lazy(y2, p.ZZZ), p.Y);
  Fq X = p.X, Y = p.Y, ZZ = p.ZZ, ZZZ = p.ZZZ;
  bool dbl = false;
  if (fe_is_zero2p(Pd)) {
    if (!fe_is_zero2p(Rd)) return G1Xyzz::identity();
    const Fq x2s = fe_sqr_hp<FqTag, false>(x2);
    Pd = fe_add2p(y2, y2);
    Rd = fe_add2p(fe_add2p(x2s, x2s), x2s);
    X = x2, Y = y2, ZZ = Fq::one(), ZZZ = Fq::one();
    dbl = true;
  }
  const Fq PP = fe_sqr_hp<FqTag, false>(Pd);
  const Fq PPP = fe_mul_lazy(Pd, PP);
  const Fq Q = fe_mul_lazy(X, PP);
  const Fq R2 = fe_sqr_hp<FqTag, false>(Rd);
  const Fq X3 = fe_sub2p(fe_sub2p(dbl ? R2 : fe_sub2p(R2, PPP), Q), Q);
  const Fq x[2] = {Rd, Y};
  const Fq y[2] = {fe_sub2p(Q, X3), fe_neg2p(PPP)};
  return {X3, fe_mul_sum(x, y), fe_mul_lazy(ZZ, PP), fe_mul_lazy(ZZZ, PPP)};
}
SV_HD G1Xyzz xyzz_canon2p(const G1Xyzz& p) {
  return {fe_canon2p(p.X), fe_canon2p(p.Y), fe_canon2p(p.ZZ), fe_canon2p(p.ZZZ)};
}
// add-2008-s in the 2p domain (both inputs in [0, 2p); the identity is exactly ZZ = 0): the bucket
// reduction chains (k_wsum, k_group_sum), canonical at their stores.
SV_HD G1Xyzz xyzz_add_2p(const G1Xyzz& p, const G1Xyzz& q) {
  if (p.is_identity()) return q;
  if (q.is_identity()) return p;
  const Fq U1 = fe_mul_lazy(p.X, q.ZZ);
  const Fq U2 = fe_mul_lazy(q.X, p.ZZ);
  const Fq S1 = fe_mul_lazy(p.Y, q.ZZZ);
  const Fq S2 = fe_mul_lazy(q.Y, p.ZZZ);
  const Fq Pd = fe_sub2p(U2, U1);
  const Fq Rd = fe_sub2p(S2, S1);
  if (fe_is_zero2p(Pd)) {
    if (fe_is_zero2p(Rd)) return xyzz_dbl(xyzz_canon2p(p));
    return G1Xyzz::identity();
  }
  const Fq PP = fe_sqr_hp<FqTag, false>(Pd);
  const Fq PPP = fe_mul_lazy(Pd, PP);
  const Fq Q = fe_mul_lazy(U1, PP);
  const Fq X3 = fe_sub2p(fe_sub2p(fe_sub2p(fe_sqr_hp<FqTag, false>(Rd), PPP), Q), Q);
  const Fq x[2] = {Rd, S1};
  const Fq y[2] = {fe_sub2p(Q, X3), fe_neg2p(PPP)};
  return {X3, fe_mul_sum(x, y), fe_mul_lazy(fe_mul_lazy(p.ZZ, q.ZZ), PP),
          fe_mul_lazy(fe_mul_lazy(p.ZZZ, q.ZZZ), PPP)};
}

// add-2008-s
SV_HD G1Xyzz xyzz_add(const G1Xyzz& p, const G1Xyzz& q) {
  if (p.is_identity()) return q;
  if (q.is_identity()) return p;
  Fq U1 = p.X * q.ZZ;
  Fq U2 = q.X * p.ZZ;
  Fq S1 = p.Y * q.ZZZ;
  Fq S2 = q.Y * p.ZZZ;
  Fq Pd = U2 - U1;
  Fq Rd = S2 - S1;
  if (Pd.is_zero()) {
    if (Rd.is_zero()) return xyzz_dbl(p);
    return G1Xyzz::identity();
  }
  Fq PP = fe_sqr_hp(Pd);
  Fq PPP = Pd * PP;
  Fq Q = U1 * PP;
  Fq X3 = fe_sqr_hp(Rd) - PPP - fe_dbl(Q);
  Fq Y3 = mul_diff(Rd, Q - X3, S1, PPP);
  return {X3, Y3, p.ZZ * q.ZZ * PP, p.ZZZ * q.ZZZ * PPP};
}

SV_HD G1Xyzz xyzz_neg(const G1Xyzz& p) { return {p.X, -p.Y, p.ZZ, p.ZZZ}; }

// Affine conversion (Fermat inversions; host/tail use only).
SV_NOINL G1Aff xyzz_to_affine(const G1Xyzz& p) {
  if (p.is_identity()) return {Fq::zero(), Fq::zero()};
  // ZZZ^-1 = 1/Z^3; x = X * ZZ^-1, y = Y * ZZZ^-1
  Fq izzz = fe_inv(p.ZZZ);
  Fq iz = izzz * p.ZZ;        // 1/Z
  Fq izz = fe_sqr(iz);        // 1/Z^2
  return {p.X * izz, p.Y * izzz};
}

// ------------------------------------------------------------------------------------------
// G2 line precomputation (host side of the decider; once per call per G2 point, as
// halo2curves' G2Prepared::from -- which the reference recomputes on every decide,
// snark-verifier/src/pcs/kzg/decider.rs:64).
// ------------------------------------------------------------------------------------------
struct G2Aff {
  Fq2 x, y;
  SV_HD bool is_identity() const { return x.is_zero() && y.is_zero(); }
};
struct G2Proj {
  Fq2 X, Y, Z;
};
struct LineCoeff {
  Fq2 c0, c3, c4;
};

SV_NOINL LineCoeff g2_doubling_step(G2Proj& T) {
  Fq two_inv = fq_const(FQ_TWO_INV);
  Fq2 a = (T.X * T.Y) * two_inv;
  Fq2 b = fq2_sqr(T.Y);
  Fq2 c = fq2_sqr(T.Z);
  Fq2 c3 = fq2_dbl(c) + c;
  Fq2 e = fq2_const(TWIST_B_C0, TWIST_B_C1) * c3;
  Fq2 f = fq2_dbl(e) + e;
  Fq2 g = (b + f) * two_inv;
  Fq2 h = fq2_sqr(T.Y + T.Z) - (b + c);
  Fq2 i = e - b;
  Fq2 j = fq2_sqr(T.X);
  Fq2 e2 = fq2_sqr(e);
  T.X = a * (b - f);
  T.Y = fq2_sqr(g) - (fq2_dbl(e2) + e2);
  T.Z = b * h;
  return {-h, fq2_dbl(j) + j, i};
}

SV_NOINL LineCoeff g2_addition_step(G2Proj& T, const G2Aff& Q) {
  Fq2 theta = T.Y - Q.y * T.Z;
  Fq2 lambda = T.X - Q.x * T.Z;
  Fq2 c = fq2_sqr(theta);
  Fq2 d = fq2_sqr(lambda);
  Fq2 e = lambda * d;
  Fq2 f = T.Z * c;
  Fq2 g = T.X * d;
  Fq2 h = e + f - fq2_dbl(g);
  T.X = lambda * h;
  T.Y = theta * (g - h) - e * T.Y;
  T.Z = T.Z * e;
  Fq2 j = theta * Q.x - lambda * Q.y;
  return {lambda, -theta, j};
}

SV_NOINL G2Aff g2_frob(const G2Aff& q) {
  return {fq2_conj(q.x) * fq2_const(TWIST_FROB_X_C0, TWIST_FROB_X_C1),
          fq2_conj(q.y) * fq2_const(TWIST_FROB_Y_C0, TWIST_FROB_Y_C1)};
}

// Fills ATE_NUM_LINES coefficients; same step order as the Miller loop below.
inline void g2_prepare(const G2Aff& Q, LineCoeff* out) {
  G2Proj T = {Q.x, Q.y, Fq2::one()};
  G2Aff negQ = {Q.x, -Q.y};
  int k = 0;
  for (int i = ATE_NAF_LEN - 2; i >= 0; i--) {
    out[k++] = g2_doubling_step(T);
    if (ATE_NAF[i] == 1) out[k++] = g2_addition_step(T, Q);
    else if (ATE_NAF[i] == -1) out[k++] = g2_addition_step(T, negQ);
  }
  G2Aff Q1 = g2_frob(Q);
  G2Aff Q2 = g2_frob(Q1);
  Q2.y = -Q2.y;
  out[k++] = g2_addition_step(T, Q1);
  out[k++] = g2_addition_step(T, Q2);
}

SV_NOINL void ell(Fq12& f, const LineCoeff& c, const G1Aff& p) {
  f = fq12_mul_by_034(f, c.c0 * p.y, c.c3 * p.x, c.c4);
}

// 2-term multi-Miller loop of the decider: prod over {(p1, L1), (p2, L2)}; identity G1 terms
// are skipped (contribute 1), as halo2curves' multi_miller_loop does.
template <class LineSrc>
SV_NOINL Fq12 miller_loop_2(const G1Aff& p1, const LineSrc& L1, const G1Aff& p2, const LineSrc& L2) {
  bool use1 = !p1.is_identity(), use2 = !p2.is_identity();
  Fq12 f = Fq12::one();
  int k = 0;
  for (int i = ATE_NAF_LEN - 1; i >= 1; i--) {
    if (i != ATE_NAF_LEN - 1) f = fq12_sqr(f);
    if (use1) ell(f, L1[k], p1);
    if (use2) ell(f, L2[k], p2);
    k++;
    if (ATE_NAF[i - 1] != 0) {
      if (use1) ell(f, L1[k], p1);
      if (use2) ell(f, L2[k], p2);
      k++;
    }
  }
  for (int s = 0; s < 2; s++) {
    if (use1) ell(f, L1[k], p1);
    if (use2) ell(f, L2[k], p2);
    k++;
  }
  return f;
}

SV_NOINL Fq12 fq12_pow_x(const Fq12& a) {  // a^BN_X, MSB first
  Fq12 r = a;
  for (int b = 61; b >= 0; b--) {  // BN_X has bit 62 as its top bit
    r = fq12_sqr(r);
    if ((BN_X >> b) & 1) r = r * a;
  }
  return r;
}

SV_NOINL Fq12 fq12_pow_small(const Fq12& a, uint32_t e) {
  Fq12 r = Fq12::one();
  bool started = false;
  for (int b = 31; b >= 0; b--) {
    if (started) r = fq12_sqr(r);
    if ((e >> b) & 1) {
      r = started ? r * a : a;
      started = true;
    }
  }
  return r;
}

SV_NOINL Fq12 final_exponentiation(const Fq12& f0) {
  // easy part: f^((p^6 - 1)(p^2 + 1))
  Fq12 f = fq12_conj(f0) * fq12_inv(f0);
  f = fq12_frob<2>(f) * f;
  // hard part: lam0 + lam1 p + lam2 p^2 + p^3 (see oracle/bn254.py final_exp_hard_chain)
  Fq12 fx = fq12_pow_x(f);
  Fq12 fx2 = fq12_pow_x(fx);
  Fq12 fx3 = fq12_pow_x(fx2);
  Fq12 fx3_36 = fq12_pow_small(fx3, 36);
  Fq12 l2 = fq12_pow_small(fx2, 6) * f;
  Fq12 l1 = fq12_conj(fx3_36 * fq12_pow_small(fx2, 18) * fq12_pow_small(fx, 12)) * f;
  Fq12 l0 = fq12_conj(fx3_36 * fq12_pow_small(fx2, 30) * fq12_pow_small(fx, 18) * fq12_sqr(f));
  return l0 * fq12_frob<1>(l1) * fq12_frob<2>(l2) * fq12_frob<3>(f);
}

}  // namespace sv
