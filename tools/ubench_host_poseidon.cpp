// Host microbenchmark (round 5): one serial t = 3 Poseidon permutation chain (create_proof's
// transcript sponge) -- the product's csrc/host_poseidon.hpp against the round-4 schedule (a copy
// passed with -DOLD_HDR=<path>), same inputs, results compared.
// Build: clang++ -O3 -std=c++17 -Isnark-verifier-axiom_amd/csrc -DOLD_HDR='"/tmp/host_poseidon_old.hpp"' \
//          tools/ubench_host_poseidon.cpp -o tools/ubench_host_poseidon
#include <chrono>
#include <cstdio>

#include "host_poseidon.hpp"
#ifdef OLD_HDR
namespace old_impl {
#define sv sv_old
#include OLD_HDR
#undef sv
}  // namespace old_impl
#endif

template <class F>
static double time_chain(F f, int iters) {
  f();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; i++) f();
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
}

int main() {
  using namespace sv::host::fr;
  E s[3] = {{{1, 2, 3, 4}}, {{5, 6, 7, 8}}, {{9, 10, 11, 0x0fffffffffffffffull}}};
  const int iters = 20000;
  const double tn = time_chain([&] { permute3(s); }, iters);
  printf("new permute3: %.3f us per permutation (state %016llx)\n", tn, (unsigned long long)s[0].l[0]);
#ifdef OLD_HDR
  {
    using namespace old_impl::sv_old::host::fr;
    old_impl::sv_old::host::fr::E o[3] = {{{1, 2, 3, 4}}, {{5, 6, 7, 8}}, {{9, 10, 11, 0x0fffffffffffffffull}}};
    const double to = time_chain([&] { old_impl::sv_old::host::fr::permute3(o); }, iters);
    printf("old permute3: %.3f us per permutation (state %016llx)\n", to, (unsigned long long)o[0].l[0]);
    bool same = true;
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 4; k++) same &= o[i].l[k] == s[i].l[k];
    printf("same states after %d chained permutations: %s\n", iters + 1, same ? "yes" : "NO");
    return same ? 0 : 1;
  }
#endif
  return 0;
}
