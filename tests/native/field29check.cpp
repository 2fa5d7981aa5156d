// Test harness (not part of libsvgpu): every operation of csrc/field29.hpp on the host, over random
// and boundary operands at the bounds the header states; prints "op inputs... output" lines (hex
// integers) for tests/test_field29.py, which checks values mod p and output bounds with Python ints.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <initializer_list>
#include <string>
#include <type_traits>

#include "curve29.hpp"

using namespace sv::r29;

static uint64_t s = 0x9E3779B97F4A7C15ull;
static int g_top = 23;
static int n_top_bits() { return g_top; }
static uint64_t rnd() {
  s ^= s << 13;
  s ^= s >> 7;
  s ^= s << 17;
  return s;
}
// a value below k p: random limbs, then csub down (k p below 2^261), or a boundary value
template <class M>
static F29<M> below(int k, int mode) {
  F29<M> r;
  if (mode == 1) return zero<M>();
  if (mode == 2) {  // k p - 1
    F29<M> kp1 = k == 1 ? kp_f<1, M>() : k == 2 ? kp_f<2, M>() : k == 4 ? kp_f<4, M>() : kp_f<6, M>();
    F29<M> one = zero<M>();
    one.v[0] = 1;
    F29<M> t = sub<1>(kp1, one);  // kp - 1 + p
    return csub<1>(t) /* value kp - 1 when k >= 1 */;
  }
  for (int i = 0; i < L; i++) r.v[i] = (uint32_t)rnd() & MASK;
  r.v[L - 1] &= (n_top_bits() == 23 ? 0x7fffffu : 0x3fffffu);  // below 2^255 (~4.4 p) or 2^254
  return r;
}
template <class M>
static void pr(const F29<M>& a) {
  printf(" ");
  for (int i = L - 1; i >= 0; i--) printf("%08x", a.v[i]);
}
// hex integer (below 2^261) -> normalized limbs
static F parse(const std::string& h) {
  F r = zero();
  int bit = 0;
  for (int k = (int)h.size() - 1; k >= 0 && h[k] != 'x'; k--, bit += 4) {
    const char c = h[k];
    const uint32_t d = c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
    r.v[bit / 29] |= (d << (bit % 29)) & MASK;
    if (bit % 29 > 25) r.v[bit / 29 + 1] |= d >> (29 - bit % 29);
  }
  return r;
}
// "madd" / "maddn" mode: stdin lines "X Y ZZ ZZZ x2 y2" (hex) -> "X3 Y3 ZZ3 ZZZ3" of
// state + (x2, y2) / state + (x2, -y2).  "maddl" / "maddln": the round-6 loop's pair -- an
// identity state takes start(x2, +-y2), any other madd_live (its doubling case replaced by dbl_start,
// its cancellation zeroing ZZ, as the loop does: the loop marks that chain empty and a stored one
// reads as the identity by ZZ == 0).
static bool g_neg = false, g_live = false;
static int madd_mode() {
  char buf[6][80];
  while (scanf("%79s %79s %79s %79s %79s %79s", buf[0], buf[1], buf[2], buf[3], buf[4], buf[5]) == 6) {
    const Xyzz st{parse(buf[0]), parse(buf[1]), parse(buf[2]), parse(buf[3])};
    Xyzz r;
    if (!g_live) {
      r = madd(st, parse(buf[4]), parse(buf[5]), g_neg);
    } else if (is_identity(st)) {
      r = start(parse(buf[4]), parse(buf[5]), g_neg);
    } else {
      // as the loop runs it: the doubling replaced by dbl_start, a cancellation zeroes ZZ
      int special = 0;
      r = madd_live(st, parse(buf[4]), parse(buf[5]), g_neg, special);
      if (special == 2) r = dbl_start(parse(buf[4]), parse(buf[5]), g_neg);
      else if (special == 1) r.ZZ = zero();
    }
    pr(r.X), pr(r.Y), pr(r.ZZ), pr(r.ZZZ);
    printf("\n");
  }
  return 0;
}

template <class M>
static int run_ops(bool fq) {
  for (int n = 0; n < 3000; n++) {
    const int mode = n < 40 ? n % 3 : 0;
    g_top = (n & 1) ? 23 : 22;
    // raw random below 2^255 (~4.4 p); the Python side knows each op's input bound and checks it
    F29<M> a = below<M>(12, mode), b = below<M>(12, (mode + 1) % 3), c = below<M>(12, mode), d = below<M>(12, (mode + 2) % 3);
    printf("mul");
    pr(a), pr(b), pr(mul(a, b));
    printf("\nmul_ilp");
    pr(a), pr(b), pr(mul_ilp(a, b));
    printf("\nsqr");
    pr(a), pr(sqr(a));
    printf("\nmul_sum2");
    pr(a), pr(b), pr(c), pr(d), pr(mul_sum2(a, b, c, d));
    {  // mul_sum3 over "constants" below p (b, d reduced)
      const F29<M> bb = csub<1>(csub<2>(csub<4>(b))), dd = csub<1>(csub<2>(csub<4>(d))), ee = csub<1>(csub<2>(csub<4>(a)));
      printf("\nmul_sum3");
      pr(a), pr(bb), pr(c), pr(dd), pr(d), pr(ee), pr(mul_sum3(a, bb, c, dd, d, ee));
    }
    printf("\nadd");
    pr(a), pr(b), pr(add(a, b));
    printf("\nsub2");
    pr(a), pr(b), pr(sub<2>(a, b));
    printf("\nsub4");
    pr(a), pr(b), pr(sub<4>(a, b));
    printf("\nsub6");
    pr(a), pr(b), pr(sub<6>(a, b));
    printf("\nsub8");
    pr(a), pr(b), pr(sub<8>(a, b));
    printf("\nsub2c6");
    pr(a), pr(b), pr(c), pr(sub_2c<6>(a, b, c));
    printf("\nmul_sub8");  // c below 8p (a csub chain bound it below 4p, then + up to 3p)
    {
      const F29<M> c8 = csub<4>(c);
      pr(a), pr(b), pr(c8), pr(mul_sub<8>(a, b, c8));
    }
    printf("\nsqr_sub2c6");  // b below 2p, c below 2p (the chain's PPP and Q)
    {
      const F29<M> b2 = csub<1>(csub<2>(csub<4>(b))), c2 = csub<1>(csub<2>(csub<4>(d)));
      pr(a), pr(b2), pr(c2), pr(sqr_sub2c<6>(a, b2, c2));
    }
    printf("\ncsub1");
    pr(a), pr(csub<1>(a));
    printf("\ncsub2");
    pr(a), pr(csub<2>(a));
    printf("\ncsub4");
    pr(a), pr(csub<4>(a));
    if constexpr (std::is_same<M, FqM29>::value) {
      printf("\nzero6 ");
      pr(a);
      printf(" %d", is_zero_mod_p_6p(a) ? 1 : 0);
      printf("\nzero10 ");
      pr(a);
      printf(" %d", is_zero_mod_p_10p(a) ? 1 : 0);
      printf("\nzero16 ");
      pr(a);
      printf(" %d", is_zero_mod_p_16p(a) ? 1 : 0);
    }
    uint32_t w[8], w2[8];
    to_words(a, w);
    F29<M> back = from_words<M>(w);
    printf("\nwords");
    pr(a), pr(back);
    // conversions (inputs below p as 8 x 32 words: a mod p computed via csub chain)
    F29<M> ar = csub<1>(csub<2>(csub<4>(a)));
    to_words(ar, w);
    F29<M> r29 = to_r29<M>(w);
    to_r32(r29, w2);
    printf("\nto_r29");
    pr(ar), pr(r29), pr(from_words<M>(w2));
    F29<M> a4 = csub<4>(a);  // below 4p when a is below 8p
    to_r32(a4, w2);
    printf("\nto_r32");
    pr(a4), pr(from_words<M>(w2));
    printf("\n");
  }
  // zero tests on exact multiples of p
  for (int k = 0; fq && k < 16; k++) {
    F m = zero();
    for (int j = 0; j < k; j++) m = sub<1>(m, zero());  // m + p
    if (k < 6) {
      printf("zero6 ");
      pr(m);
      printf(" %d\n", is_zero_mod_p_6p(m) ? 1 : 0);
    }
    if (k < 10) {
      printf("zero10 ");
      pr(m);
      printf(" %d\n", is_zero_mod_p_10p(m) ? 1 : 0);
    }
    printf("zero16 ");
    pr(m);
    printf(" %d\n", is_zero_mod_p_16p(m) ? 1 : 0);
    // neighbours of k p: limb 0 matches a multiple's, the value does not
    for (int d : {-1, 1}) {
      F n = m;
      n.v[L - 1] += (uint32_t)d;  // k p +- 2^232: the top limb moves, limb 0 stays
      if (k == 0 && d < 0) continue;
      printf("zero16 ");
      pr(n);
      printf(" %d\n", is_zero_mod_p_16p(n) ? 1 : 0);
    }
  }
  return 0;
}

// "xadd" mode: stdin lines "X Y ZZ ZZZ X' Y' ZZ' ZZZ'" (hex) -> "X3 Y3 ZZ3 ZZZ3"
static int xadd_mode() {
  char b[8][80];
  while (scanf("%79s %79s %79s %79s %79s %79s %79s %79s", b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]) == 8) {
    const Xyzz p{parse(b[0]), parse(b[1]), parse(b[2]), parse(b[3])};
    const Xyzz q{parse(b[4]), parse(b[5]), parse(b[6]), parse(b[7])};
    const Xyzz r = sv::r29::add(p, q);
    pr(r.X), pr(r.Y), pr(r.ZZ), pr(r.ZZZ);
    printf("\n");
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "madd")) return madd_mode();
  if (argc > 1 && !strcmp(argv[1], "maddn")) return g_neg = true, madd_mode();
  if (argc > 1 && !strcmp(argv[1], "maddl")) return g_live = true, madd_mode();
  if (argc > 1 && !strcmp(argv[1], "maddln")) return g_live = g_neg = true, madd_mode();
  if (argc > 1 && !strcmp(argv[1], "xadd")) return xadd_mode();
  const bool fr = argc > 1 && !strcmp(argv[1], "fr");  // the same checks over Fr (FrM29)
  return fr ? run_ops<FrM29>(false) : run_ops<FqM29>(true);
}

