// Host check: per-lane w-basis Fq12 ops (fq12_lanes.hpp) == tower ops (field.hpp).
#include "fq12_lanes.hpp"
#include <cstdio>
#include <random>
using namespace sv;
static Fq rnd(std::mt19937_64& g) { Fq r; for (int i = 0; i < 8; i++) r.v[i] = (uint32_t)g(); r.v[7] &= 0x0fffffff; return fe_to_mont(r); }
static Fq12 rnd12(std::mt19937_64& g) { Fq12 f; for (int k = 0; k < 6; k++) { tower_coeff(f, k).c0 = rnd(g); tower_coeff(f, k).c1 = rnd(g); } return f; }
int main() {
  std::mt19937_64 g(42);
  static const SqrTerm tab[6][4] = SV_SQR_TERMS;
  int bad = 0;
  for (int it = 0; it < 20; it++) {
    Fq12 a = rnd12(g), b = rnd12(g);
    Fq2 A[6], B[6];
    for (int k = 0; k < 6; k++) { A[k] = tower_coeff(a, k); B[k] = tower_coeff(b, k); }
    Fq12 m = a * b, s = fq12_sqr(a);
    Fq2 c0 = {rnd(g), rnd(g)}, c3 = {rnd(g), rnd(g)}, c4 = {rnd(g), rnd(g)};
    Fq12 l = fq12_mul_by_034(a, c0, c3, c4);
    for (int k = 0; k < 6; k++) {
      bad += !(w_mul_lane(A, B, k) == tower_coeff(m, k));
      bad += !(w_sqr_lane(A, k, tab) == tower_coeff(s, k));
      bad += !(w_line_lane(A, c0, c3, c4, k) == tower_coeff(l, k));
    }
  }
  printf("lane ops mismatches: %d\n", bad);
  return bad != 0;
}
