// Fq12 spread over 6 lanes: f = sum_{k<6} g_k w^k with g_k in Fq2 and w^6 = xi = 9 + u.
//
// The tower basis {1, v, v^2, w, vw, v^2 w} of curve.hpp is exactly {w^0, w^2, w^4, w^1, w^3, w^5},
// so lane k of a group holds tower coefficient TOWER_OF[k] and no conversion is ever needed.  Each
// function below returns lane k's coefficient of the result from the group's full operands (read
// from LDS on the device, from arrays in the host unit check):
//   w_mul_lane     6 Fq2 products per lane   (vs 54 Fq muls for one lane doing the whole Fq12 mul)
//   w_sqr_lane     <= 4 Fq2 products per lane (pair table below)
//   w_line_lane    3 Fq2 products: f * (l0 + l1 w + l3 w^3), the sparse D-type line
//   w_frob_lane    1 Fq2 product (conj^n(g_k) * xi^(k (p^n - 1)/6))
#pragma once
#include "field.hpp"

namespace sv {

// w^k <-> tower slot: k = 0..5 -> (c0.c0, c1.c0, c0.c1, c1.c1, c0.c2, c1.c2)
SV_HD const Fq2& tower_coeff(const Fq12& f, int k) {
  const Fq6& h = (k & 1) ? f.c1 : f.c0;
  const int i = k >> 1;
  return i == 0 ? h.c0 : (i == 1 ? h.c1 : h.c2);
}
SV_HD Fq2& tower_coeff(Fq12& f, int k) {
  Fq6& h = (k & 1) ? f.c1 : f.c0;
  const int i = k >> 1;
  return i == 0 ? h.c0 : (i == 1 ? h.c1 : h.c2);
}

// r_k = sum_i a_i b_{k-i}, wrapped terms (i > k) multiplied by xi
SV_HD Fq2 w_mul_lane(const Fq2* a, const Fq2* b, int k) {
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const int j = k - i;
    const Fq2 p = a[i] * b[j < 0 ? j + 6 : j];
    if (j >= 0) lo = lo + p;
    else hi = hi + p;
  }
  return lo + fq2_mul_xi(hi);
}

// Squaring: lane k sums over unordered pairs {i, j}, i + j = k (mod 6); a pair counts twice when
// i != j, and gets a factor xi when i + j >= 6.  Four slots per lane (odd k use three).
struct SqrTerm {
  int8_t i, j, dbl, xi;
};
#define SV_SQR_TERMS                                                                               \
  {{{0, 0, 0, 0}, {3, 3, 0, 1}, {1, 5, 1, 1}, {2, 4, 1, 1}},                                       \
   {{0, 1, 1, 0}, {2, 5, 1, 1}, {3, 4, 1, 1}, {-1, -1, 0, 0}},                                     \
   {{1, 1, 0, 0}, {0, 2, 1, 0}, {4, 4, 0, 1}, {3, 5, 1, 1}},                                       \
   {{0, 3, 1, 0}, {1, 2, 1, 0}, {4, 5, 1, 1}, {-1, -1, 0, 0}},                                     \
   {{2, 2, 0, 0}, {0, 4, 1, 0}, {1, 3, 1, 0}, {5, 5, 0, 1}},                                       \
   {{0, 5, 1, 0}, {1, 4, 1, 0}, {2, 3, 1, 0}, {-1, -1, 0, 0}}}

SV_HD Fq2 w_sqr_lane(const Fq2* a, int k, const SqrTerm (*tab)[4]) {
  Fq2 lo = Fq2::zero(), hi = Fq2::zero();
#pragma unroll
  for (int s = 0; s < 4; s++) {
    const SqrTerm t = tab[k][s];
    if (t.i < 0) continue;
    Fq2 p = a[t.i] * a[t.j];
    if (t.dbl) p = p + p;
    if (t.xi) hi = hi + p;
    else lo = lo + p;
  }
  return lo + fq2_mul_xi(hi);
}

// f * (l0 + l1 w + l3 w^3)
SV_HD Fq2 w_line_lane(const Fq2* g, const Fq2& l0, const Fq2& l1, const Fq2& l3, int k) {
  Fq2 lo = g[k] * l0;
  Fq2 hi = Fq2::zero();
  const Fq2 p1 = g[k >= 1 ? k - 1 : k + 5] * l1;
  if (k >= 1) lo = lo + p1;
  else hi = hi + p1;
  const Fq2 p3 = g[k >= 3 ? k - 3 : k + 3] * l3;
  if (k >= 3) lo = lo + p3;
  else hi = hi + p3;
  return lo + fq2_mul_xi(hi);
}

}  // namespace sv
