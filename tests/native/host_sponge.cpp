// Test harness (not part of libsvgpu): drives the product's host Poseidon transcript
// (csrc/host_poseidon.hpp, used by sv_bn254_kzg_create_proof) so a CPU test can compare it with
// oracle/poseidon.py.  stdin: "t0 t1 t2" canonical hex state (or "-" = fresh), then one canonical
// hex Fr element per line; stdout: the squeezed challenge and the state after, canonical hex.
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "host_poseidon.hpp"

using namespace sv::host::fr;

static E parse(const std::string& h) {
  E e{{0, 0, 0, 0}};
  std::string s = h.substr(h.rfind('x') == std::string::npos ? 0 : h.rfind('x') + 1);
  for (char c : s) {
    const int v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    for (int i = 3; i > 0; i--) e.l[i] = (e.l[i] << 4) | (e.l[i - 1] >> 60);
    e.l[0] = (e.l[0] << 4) | (uint64_t)v;
  }
  return e;
}

static void print(const E& e) { printf("%016llx%016llx%016llx%016llx", (unsigned long long)e.l[3],
                                       (unsigned long long)e.l[2], (unsigned long long)e.l[1],
                                       (unsigned long long)e.l[0]); }

int main() {
  Sponge3 sp;
  std::string a, b, c;
  std::cin >> a;
  if (a != "-") {
    std::cin >> b >> c;
    sp.st[0] = to_mont(parse(a)), sp.st[1] = to_mont(parse(b)), sp.st[2] = to_mont(parse(c));
  }
  std::string x;
  while (std::cin >> x) sp.update(to_mont(parse(x)));
  const E r = from_mont(sp.squeeze());
  print(r);
  for (int k = 0; k < 3; k++) printf(" "), print(from_mont(sp.st[k]));
  printf("\n");
  return 0;
}
