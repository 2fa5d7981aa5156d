// Host-side check of the device templates (field.hpp / curve.hpp) against oracle/bn254.py.
// Build: g++ -O2 -std=c++17 -I snark-verifier-axiom_amd/csrc tools/hostcheck.cpp -o /tmp/hostcheck
#include "curve.hpp"
#include <cstdio>
#include <cstring>
using namespace sv;
static Fq from_hex(const char* h) {  // big-endian hex, canonical -> Montgomery
  Fq r = Fq::zero();
  int n = strlen(h);
  for (int i = 0; i < n; i++) {
    int c = h[n - 1 - i];
    int v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    r.v[i / 8] |= (uint32_t)v << (4 * (i % 8));
  }
  return fe_to_mont(r);
}
static void print_fq(const Fq& a) {
  Fq c = fe_from_mont(a);
  for (int i = 7; i >= 0; i--) printf("%08x", c.v[i]);
  printf("\n");
}
int main(int argc, char** argv) {
  // G1 = (1,2), G2 standard generator
  G1Aff g1 = {from_hex("1"), from_hex("2")};
  G2Aff g2 = {{from_hex("1800deef121f1e76426a00665e5c4479674322d4f75edadd46debd5cd992f6ed"),
               from_hex("198e9393920d483a7260bfb731fb5d25f1aa493335a9e71297e485b7aef312c2")},
              {from_hex("12c85ea5db8c6deb4aab71808dcb408fe3d1e7690c43d37b4ce6cc0166fa7daa"),
               from_hex("090689d0585ff075ec9e99ad690c3395bc4b313370b38ef355acdadcd122975b")}};
  static LineCoeff L[ATE_NUM_LINES];
  g2_prepare(g2, L);
  G1Aff none = {Fq::zero(), Fq::zero()};
  Fq12 f = miller_loop_2(g1, L, none, L);
  Fq12 e = final_exponentiation(f);
  // print Gt in c0.c0.c0, c0.c0.c1, ... order
  const Fq6* c6[2] = {&e.c0, &e.c1};
  for (int i = 0; i < 2; i++) {
    const Fq2* c2[3] = {&c6[i]->c0, &c6[i]->c1, &c6[i]->c2};
    for (int j = 0; j < 3; j++) { print_fq(c2[j]->c0); print_fq(c2[j]->c1); }
  }
  // G1: 2G via dbl, 3G via madd, G + (-G)
  G1Xyzz a = G1Xyzz::from_affine(g1);
  G1Xyzz d = xyzz_dbl(a);
  G1Xyzz t = xyzz_madd(d, g1.x, g1.y);
  G1Aff t3 = xyzz_to_affine(t);
  print_fq(t3.x); print_fq(t3.y);
  G1Xyzz z = xyzz_madd(a, g1.x, -g1.y);
  printf("G+(-G) identity: %d\n", (int)z.is_identity());
  G1Xyzz dd = xyzz_madd(a, g1.x, g1.y);  // G + G via madd special case
  G1Xyzz s = xyzz_add(dd, t);  // 2G + 3G = 5G
  G1Aff s5 = xyzz_to_affine(s);
  print_fq(s5.x); print_fq(s5.y);
  return 0;
}
