// XYZZ mixed addition over field29.hpp's 9 x 29-bit limbs (round 4): k_accumulate's inner step.
//
// Bounds (field29.hpp's lazy contract), kept by every function here:
//   state  X < 4p, Y < 2p, ZZ < 2p, ZZZ < 2p; the identity is exactly all-zero limbs (ZZ == 0: a
//          non-identity state never has ZZ = 0 mod p, since ZZ3 = ZZ PP and PP != 0 mod p);
//          madd's chain state (round 5) lets X reach 8p: its X3 skips the conditional subtraction,
//          and whoever stores the chain's sum brings X below 4p (k_accumulate: csub<4> at a
//          segment's end, AccChain<true>::out);
//   point  x2, y2 below 2p (R' form), never the identity (callers skip it).
// The formulas are madd-2008-s / mdbl-2008-s, as xyzz_madd_2p / xyzz_mdbl in curve.hpp.
#pragma once
#include "field29.hpp"

namespace sv {
namespace r29 {

struct Xyzz {
  F X, Y, ZZ, ZZZ;
};

SV29_HD F one() {  // R' mod p
  F r;
  constexpr uint32_t O[L] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x14c0419u, 0xaa36fb9u,
                             0x1d4240ceu, 0x11d54c07u, 0x52ac7a8u,  0x00dc836u};
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = O[i];
  return r;
}
SV29_HD Xyzz identity() { return {zero(), zero(), zero(), zero()}; }
SV29_HD bool is_identity(const Xyzz& p) { return is_zero(p.ZZ); }

// p + (x2, y2).  The doubling case (p = (x2, y2)) runs through the same products: mdbl's U = 2 y2,
// V = U^2, W = U V, S = x2 V, M = 3 x2^2 are the addition's Pd, PP, PPP, Q (with X = x2) and Rd, and
// X3 = M^2 - 2S, Y3 = M (S - X3) - y2 W, ZZ3 = V, ZZZ3 = W its outputs with (X, Y, ZZ, ZZZ) =
// (x2, y2, 1, 1) and no PPP term in X3 -- the rare branch only sets operands (one extra square),
// so the chain holds no registers for a separate doubling (k_accumulate fits 128 VGPRs).
// p + (x2, neg ? -y2 : y2): the sign is applied to S2 = y2 ZZZ (one pass: Rd = +-S2 - Y + 4p)
// instead of negating y2 before the addition (a subtraction pass and a select for every entry)
SV29_HD Xyzz madd(const Xyzz& p, const F& x2, const F& y2, bool neg) {
  if (is_identity(p)) return {x2, neg ? sub<2>(zero(), y2) : y2, one(), one()};
  F Pd = sub<8>(mul(x2, p.ZZ), p.X);                 // U2 - X: < 10p (state X < 8p)
  F Rd = sub_sgn<4>(mul(y2, p.ZZZ), neg, p.Y);       // +-S2 - Y + 4p: < 6p
  F X = p.X, Y = p.Y, ZZ = p.ZZ, ZZZ = p.ZZZ;
  bool dbl = false;
  if (is_zero_mod_p_10p(Pd)) {
    if (!is_zero_mod_p_6p(Rd)) return identity();
    const F x2s = sqr(x2), ys = neg ? sub<2>(zero(), y2) : y2;
    Pd = add(ys, ys);               // < 4p
    Rd = add(add(x2s, x2s), x2s);   // < 6p
    X = x2, Y = ys, ZZ = one(), ZZZ = one();
    dbl = true;
  }
  // sqr / mul take inputs below 12p: Pd < 10p, X < 8p
  const F PP = sqr(Pd), PPP = mul(Pd, PP), Q = mul(X, PP), R2 = sqr(Rd);  // < 2p
  // X3 = R2 [- PPP] - 2Q + 6p in one pass: in (0, 8p), left there (the next madd's sub<8> and
  // mul take it; a stored sum is brought below 4p by its writer)
  const F X3 = sub_2c<6>(R2, dbl ? zero() : PPP, Q);
  // Y3 = Rd (Q - X3) - Y PPP, one reduction: Rd < 6p, Q + 8p - X3 < 10p, Y < 2p, 2p - PPP < 2p:
  // 60p^2 + 4p^2 below p R' = 169.6p^2, so the output is below 2p
  const F Y3 = mul_sum2(Rd, sub<8>(Q, X3), Y, sub<2>(zero(), PPP));
  return {X3, Y3, mul(ZZ, PP), mul(ZZZ, PPP)};
}
SV29_HD Xyzz madd(const Xyzz& p, const F& x2, const F& y2) { return madd(p, x2, y2, false); }

// Round 6: the bucket chain's two halves of madd for a loop that never lets its state be the
// identity (k_accumulate, SVGPU_ACC_LOOP=1): a segment starts with its first point (start) in the
// loop's divergent segment-end block, and the per-entry step (madd_live) has no identity test and
// no identity-valued exit -- the merges those needed cost ~100 VALU instructions per entry (register
// copies, 36 zeroing moves, the identity branch).  P + (-P) sets `cancel` and leaves a meaningless
// state: the caller marks the chain empty and restarts it with its next point.
// (x2, -y2) starts as (x2, y2, 1, -1): y = Y / ZZZ, and ZZ^3 = ZZZ^2 still holds (Z = -1), so the sign
// is a choice between two constants for ZZZ instead of a subtraction pass over y2
SV29_HD F neg_one() {  // p - R' mod p
  F r;
  constexpr uint32_t O[L] = {0x3003126u, 0xce8395eu, 0x420727bu, 0x1891eb7u, 0xae269bfu,
                             0x598fff2u, 0xed19539u, 0x9315e8bu, 0x229c18u};
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = O[i];
  return r;
}
SV29_HD Xyzz start(const F& x2, const F& y2, bool neg) { return {x2, y2, one(), neg ? neg_one() : one()}; }
// special (round 6, cont.): 0 the common case; 1 P + (-P), whose result is meaningless except that
// the caller marks the chain empty and zeroes ZZ (a stored empty chain reads as the identity); 2 the
// doubling P + P, whose result the caller replaces by dbl_start.  Both rare cases leave madd_live's
// products running on as garbage.
SV29_HD Xyzz madd_live(const Xyzz& p, const F& x2, const F& y2, bool neg, int& special) {
  const F Pd = mul_sub<8>(x2, p.ZZ, p.X);                  // U2 - X + 8p, fused: < 10p (state X < 8p)
  const F Rd = sub_sgn<4>(mul(y2, p.ZZZ), neg, p.Y);       // +-S2 - Y + 4p: < 6p
  if (is_zero_mod_p_10p(Pd)) special = is_zero_mod_p_6p(Rd) ? 2 : 1;
  const F PP = sqr(Pd), PPP = mul(Pd, PP), Q = mul(p.X, PP);  // < 2p
  // X3 = Rd^2 - PPP - 2Q + 6p in the square's high columns: in (0, 8p)
  const F X3 = sqr_sub2c<6>(Rd, PPP, Q);
  const F Y3 = mul_sum2(Rd, sub<8>(Q, X3), p.Y, sub<2>(zero(), PPP));
  return {X3, Y3, mul(p.ZZ, PP), mul(p.ZZZ, PPP)};
}
// 2 (x2, +-y2) as a chain state (madd_live's special == 2): dbl-2008-s-1 at Z = 1 -- the same
// products as the addition with Pd = 2y, Rd = 3x^2, U1 = x, S1 = y and no PPP term in X3; ZZ3 = PP,
// ZZZ3 = PPP (ZZ = ZZZ = 1).  Bounds as madd_live's: X3 < 8p, the rest < 2p.
SV29_HD Xyzz dbl_start(const F& x2, const F& y2, bool neg) {
  const F ys = neg ? sub<2>(zero(), y2) : y2;  // < 2p (y2 < 2p)
  const F x2s = sqr(x2);
  const F Pd = add(ys, ys);               // < 4p
  const F Rd = add(add(x2s, x2s), x2s);   // < 6p
  const F PP = sqr(Pd), PPP = mul(Pd, PP), Q = mul(x2, PP);
  const F X3 = sqr_sub2c<6>(Rd, zero(), Q);
  const F Y3 = mul_sum2(Rd, sub<8>(Q, X3), ys, sub<2>(zero(), PPP));
  return {X3, Y3, PP, PPP};
}

// p + q, both XYZZ states (bounds as above; either may be the identity).  add-2008-s; the
// doubling case (p = q) runs through the same products as in madd: dbl-2008-s-1's U = 2Y, M = 3X²,
// S = X V, ZZ3 = V ZZ, ZZZ3 = W ZZZ are the addition's Pd, Rd, Q, ZZ3, ZZZ3 with U1 = X, S1 = Y and
// q's ZZ, ZZZ taken as 1, and no PPP term in X3.
SV29_HD Xyzz add(const Xyzz& p, const Xyzz& q) {
  if (is_identity(p)) return q;
  if (is_identity(q)) return p;
  F U1 = mul(p.X, q.ZZ), S1 = mul(p.Y, q.ZZZ);                  // < 2p
  F Pd = sub<2>(mul(q.X, p.ZZ), U1), Rd = sub<2>(mul(q.Y, p.ZZZ), S1);  // < 4p
  F qZZ = q.ZZ, qZZZ = q.ZZZ;
  bool dbl = false;
  if (is_zero_mod_p_6p(Pd)) {
    if (!is_zero_mod_p_6p(Rd)) return identity();
    const F x2 = sqr(p.X);
    Pd = add(p.Y, p.Y);          // < 4p
    Rd = add(add(x2, x2), x2);   // < 6p
    U1 = p.X, S1 = p.Y, qZZ = one(), qZZZ = one();
    dbl = true;
  }
  const F PP = sqr(Pd), PPP = mul(Pd, PP), Q = mul(U1, PP), R2 = sqr(Rd);  // < 2p (U1 < 4p)
  const F X3 = csub<4>(sub<4>(dbl ? R2 : sub<2>(R2, PPP), add(Q, Q)));
  const F Y3 = mul_sum2(Rd, sub<4>(Q, X3), S1, sub<2>(zero(), PPP));
  return {X3, Y3, mul(mul(p.ZZ, qZZ), PP), mul(mul(p.ZZZ, qZZZ), PPP)};
}

}  // namespace r29
}  // namespace sv
