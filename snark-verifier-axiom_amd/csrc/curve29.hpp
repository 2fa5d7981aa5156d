// XYZZ mixed addition over field29.hpp's 9 x 29-bit limbs (round 4): k_accumulate's inner step.
//
// Bounds (field29.hpp's lazy contract), kept by every function here:
//   state  X < 4p, Y < 2p, ZZ < 2p, ZZZ < 2p; the identity is exactly all-zero limbs (ZZ == 0: a
//          non-identity state never has ZZ = 0 mod p, since ZZ3 = ZZ PP and PP != 0 mod p);
//   point  x2, y2 below 2p (R' form), never the identity (callers skip it).
// The formulas are add-2008-s / mdbl-2008-s, as xyzz_madd_2p / xyzz_mdbl in curve.hpp.
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

// 2 (x, y) for an affine point (x, y below 2p)
SV29_HD Xyzz mdbl(const F& x, const F& y) {
  const F U = add(y, y);                        // < 4p
  const F V = sqr(U), W = mul(U, V), S = mul(x, V);  // < 2p
  const F x2 = sqr(x);
  const F M = add(add(x2, x2), x2);             // < 6p
  const F X3 = csub<4>(sub<4>(sqr(M), add(S, S)));  // sqr(M) + 4p - 2S < 6p -> < 4p
  const F Y3 = mul_sum2(M, sub<4>(S, X3), W, sub<2>(zero(), y));  // M (S - X3) - W y: inputs < 6p
  return {X3, Y3, V, W};
}

// p + (x2, y2)
SV29_HD Xyzz madd(const Xyzz& p, const F& x2, const F& y2) {
  if (is_identity(p)) return {x2, y2, one(), one()};
  const F U2 = mul(x2, p.ZZ), S2 = mul(y2, p.ZZZ);  // < 2p
  const F Pd = sub<4>(U2, p.X);  // < 6p
  const F Rd = sub<2>(S2, p.Y);  // < 4p
  if (is_zero_mod_p_6p(Pd)) {
    if (is_zero_mod_p_6p(Rd)) return mdbl(x2, y2);
    return identity();
  }
  const F PP = sqr(Pd), PPP = mul(Pd, PP), Q = mul(p.X, PP), R2 = sqr(Rd);  // < 2p
  const F X3 = csub<4>(sub<4>(sub<2>(R2, PPP), add(Q, Q)));  // (R2 + 2p - PPP) + 4p - 2Q < 8p -> < 4p
  // Y3 = Rd (Q - X3) - Y PPP, one reduction: inputs Rd < 4p, Q + 4p - X3 < 6p, Y < 2p, 2p - PPP
  const F Y3 = mul_sum2(Rd, sub<4>(Q, X3), p.Y, sub<2>(zero(), PPP));
  return {X3, Y3, mul(p.ZZ, PP), mul(p.ZZZ, PPP)};
}

}  // namespace r29
}  // namespace sv
