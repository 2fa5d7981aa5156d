// Host check of the divsteps inversion (field.hpp fe_inv) against the binary EEA (fe_inv_eea) and
// a * a^-1 == 1, on random and edge inputs for both fields.
// Build: g++ -O2 -std=c++17 -I snark-verifier-axiom_amd/csrc tools/hostcheck_inv.cpp -o /tmp/hostcheck_inv
#include "field.hpp"
#include <cstdio>
#include <random>
using namespace sv;
template <class M>
static int run(const char* name, int n) {
  std::mt19937_64 rng(7);
  int bad = 0;
  for (int it = 0; it < n; it++) {
    Fe<M> a;
    for (int i = 0; i < 8; i++) a.v[i] = (uint32_t)rng();
    if (it < 8) {  // edges: 1, 2, m-1, m-2, small, top bits
      for (int i = 0; i < 8; i++) a.v[i] = 0;
      if (it == 0) a.v[0] = 1;
      if (it == 1) a.v[0] = 2;
      if (it == 2 || it == 3) for (int i = 0; i < 8; i++) a.v[i] = M::p(i) - (i == 0 ? (it == 2 ? 1 : 2) : 0);
      if (it == 4) a.v[0] = 0x3fffffff;
      if (it == 5) a.v[7] = 1;
      if (it == 6) a.v[3] = 0x80000000u;
      if (it == 7) a.v[0] = 3;
    }
    a.v[7] &= 0x3fffffff;
    if (!a.is_reduced() || a.is_zero()) continue;
    Fe<M> x = fe_inv(a), y = fe_inv_eea(a);
    Fe<M> one = a * x;
    if (!(x == y) || !(one == Fe<M>::one())) {
      if (bad < 5) printf("%s mismatch at %d\n", name, it);
      bad++;
    }
  }
  printf("%s: %d inputs, %d bad\n", name, n, bad);
  return bad;
}
int main() { return run<FqTag>("Fq", 200000) + run<FrTag>("Fr", 200000) ? 1 : 0; }
