// Host-side BN254 G1 arithmetic with 4 x 64-bit limbs (unsigned __int128 products).
//
// Product code (not the oracle): the Pippenger pipeline ends with O(256) serial point operations
// -- the Horner combination of the per-window / per-level partial sums and the fold of per-GPU
// partials -- which a single GPU lane would run at ~1 us per field multiply (measured, see
// DESIGN.md), so libsvgpu does that short serial tail here instead.  The Montgomery layout
// (value * 2^256 mod p, little-endian) is byte-identical to the device's 8 x 32-bit limbs.
#pragma once
#include <cstdint>
#include <cstring>

namespace sv {
namespace host {

typedef unsigned __int128 u128;

struct F {
  uint64_t l[4];
};

static constexpr uint64_t P64[4] = {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull,
                                    0xb85045b68181585dull, 0x30644e72e131a029ull};
static constexpr uint64_t NP64 = 0x87d20782e4866389ull;  // -p^-1 mod 2^64
static constexpr uint64_t ONE64[4] = {0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull,
                                      0x666ea36f7879462cull, 0x0e0a77c19a07df2full};
static constexpr uint64_t R2_64[4] = {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull,
                                      0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full};

inline F f_zero() { return F{{0, 0, 0, 0}}; }
inline F f_one() { return F{{ONE64[0], ONE64[1], ONE64[2], ONE64[3]}}; }
inline bool f_is_zero(const F& a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3]) == 0; }
inline bool f_eq(const F& a, const F& b) {
  return ((a.l[0] ^ b.l[0]) | (a.l[1] ^ b.l[1]) | (a.l[2] ^ b.l[2]) | (a.l[3] ^ b.l[3])) == 0;
}

inline void f_cond_sub_p(uint64_t t[4], uint64_t carry, F& r) {
  uint64_t d[4];
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)t[i] - P64[i] - br;
    d[i] = (uint64_t)s;
    br = (s >> 127) & 1;
  }
  bool ge = carry || !br;
  for (int i = 0; i < 4; i++) r.l[i] = ge ? d[i] : t[i];
}

inline F f_add(const F& a, const F& b) {
  uint64_t t[4];
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[i] + b.l[i] + c;
    t[i] = (uint64_t)s;
    c = s >> 64;
  }
  F r;
  f_cond_sub_p(t, (uint64_t)c, r);
  return r;
}

inline F f_sub(const F& a, const F& b) {
  uint64_t t[4];
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[i] - b.l[i] - br;
    t[i] = (uint64_t)s;
    br = (s >> 127) & 1;
  }
  F r;
  if (br) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      u128 s = (u128)t[i] + P64[i] + c;
      r.l[i] = (uint64_t)s;
      c = s >> 64;
    }
  } else {
    for (int i = 0; i < 4; i++) r.l[i] = t[i];
  }
  return r;
}

inline F f_neg(const F& a) { return f_sub(f_zero(), a); }

inline F f_mul(const F& a, const F& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = s >> 64;
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    uint64_t m = t[0] * NP64;
    s = (u128)m * P64[0] + t[0];
    c = s >> 64;
    for (int j = 1; j < 4; j++) {
      s = (u128)m * P64[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = s >> 64;
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  F r;
  f_cond_sub_p(t, t[4], r);
  return r;
}

inline F f_sqr(const F& a) { return f_mul(a, a); }
inline F f_dbl(const F& a) { return f_add(a, a); }

inline F f_to_mont(const F& a) { return f_mul(a, F{{R2_64[0], R2_64[1], R2_64[2], R2_64[3]}}); }
inline F f_from_mont(const F& a) { return f_mul(a, F{{1, 0, 0, 0}}); }

inline F f_inv(const F& a) {
  uint64_t e[4] = {P64[0] - 2, P64[1], P64[2], P64[3]};
  F r = f_one();
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = f_sqr(r);
      if ((e[i] >> b) & 1) r = f_mul(r, a);
    }
  return r;
}

inline bool f_is_reduced(const F& a, const uint64_t (&mod)[4] = P64) {
  for (int i = 3; i >= 0; i--) {
    if (a.l[i] < mod[i]) return true;
    if (a.l[i] > mod[i]) return false;
  }
  return false;
}

// scalar-field order r (Fr), for validating host-side scalar inputs
static constexpr uint64_t R64[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull,
                                    0xb85045b68181585dull, 0x30644e72e131a029ull};

// XYZZ point (Montgomery), identity ZZ = 0.  Layout identical to device sv::G1Xyzz.
struct Xyzz {
  F X, Y, ZZ, ZZZ;
};

inline Xyzz x_identity() { return Xyzz{f_zero(), f_zero(), f_zero(), f_zero()}; }
inline bool x_is_identity(const Xyzz& p) { return f_is_zero(p.ZZ); }

inline Xyzz x_dbl(const Xyzz& p) {
  if (x_is_identity(p)) return p;
  F U = f_dbl(p.Y), V = f_sqr(U), W = f_mul(U, V), S = f_mul(p.X, V);
  F X2 = f_sqr(p.X), M = f_add(f_dbl(X2), X2);
  F X3 = f_sub(f_sqr(M), f_dbl(S));
  F Y3 = f_sub(f_mul(M, f_sub(S, X3)), f_mul(W, p.Y));
  return Xyzz{X3, Y3, f_mul(V, p.ZZ), f_mul(W, p.ZZZ)};
}

inline Xyzz x_add(const Xyzz& p, const Xyzz& q) {
  if (x_is_identity(p)) return q;
  if (x_is_identity(q)) return p;
  F U1 = f_mul(p.X, q.ZZ), U2 = f_mul(q.X, p.ZZ);
  F S1 = f_mul(p.Y, q.ZZZ), S2 = f_mul(q.Y, p.ZZZ);
  F Pd = f_sub(U2, U1), Rd = f_sub(S2, S1);
  if (f_is_zero(Pd)) {
    if (f_is_zero(Rd)) return x_dbl(p);
    return x_identity();
  }
  F PP = f_sqr(Pd), PPP = f_mul(Pd, PP), Q = f_mul(U1, PP);
  F X3 = f_sub(f_sub(f_sqr(Rd), PPP), f_dbl(Q));
  F Y3 = f_sub(f_mul(Rd, f_sub(Q, X3)), f_mul(S1, PPP));
  return Xyzz{X3, Y3, f_mul(f_mul(p.ZZ, q.ZZ), PP), f_mul(f_mul(p.ZZZ, q.ZZZ), PPP)};
}

// affine (Montgomery) out; identity -> (0,0)
inline void x_to_affine(const Xyzz& p, F& x, F& y) {
  if (x_is_identity(p)) {
    x = f_zero();
    y = f_zero();
    return;
  }
  F izzz = f_inv(p.ZZZ);
  F iz = f_mul(izzz, p.ZZ);
  F izz = f_sqr(iz);
  x = f_mul(p.X, izz);
  y = f_mul(p.Y, izzz);
}

// Jacobian (x = X/Z^2, y = Y/Z^3) <-> XYZZ.   XYZZ(X, Y, ZZ, ZZZ) == Jacobian(X*ZZ*ZZZ^2 ... ) is
// avoided: a Jacobian point is XYZZ with ZZ = Z^2, ZZZ = Z^3.
inline Xyzz x_from_jacobian(const F& X, const F& Y, const F& Z) {
  if (f_is_zero(Z)) return x_identity();
  F ZZ = f_sqr(Z);
  return Xyzz{X, Y, ZZ, f_mul(ZZ, Z)};
}
// XYZZ -> Jacobian with Z = ZZZ / ZZ... needs an inversion; instead scale: Z' = ZZZ * ZZ^-1 is
// avoided by choosing Z' = ZZ * ZZZ:  X' = X * ZZ * ZZZ^2,  Y' = Y * ZZ^3 * ZZZ^2.
inline void x_to_jacobian(const Xyzz& p, F& X, F& Y, F& Z) {
  if (x_is_identity(p)) {
    X = f_one();
    Y = f_one();
    Z = f_zero();
    return;
  }
  F zzz2 = f_sqr(p.ZZZ);
  F zz3 = f_mul(f_sqr(p.ZZ), p.ZZ);
  Z = f_mul(p.ZZ, p.ZZZ);
  X = f_mul(f_mul(p.X, p.ZZ), zzz2);
  Y = f_mul(f_mul(p.Y, zz3), zzz2);
}

}  // namespace host
}  // namespace sv
