// Per-op latency of the decider's lane engine (one wave per accumulator group, as k_decide_lanes).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/ubench_decops.hip \
//          snark-verifier-axiom_amd/csrc/runtime.cpp -o tools/ubench_decops
#include "../snark-verifier-axiom_amd/csrc/decider.hip"

#include <cstdio>

using namespace sv;

template <int OP>
__global__ void __launch_bounds__(64) k_op(int iters, Fq2* out) {
  constexpr int S = 8, GL = 64;
  __shared__ Fq2 sh[12];
  const int lane = threadIdx.x;
  const bool active = lane < 6 * S;
  const int k = active ? lane / S : 5, sub = active ? lane % S : 0;
  Grp G{sh, sh + 6, nullptr, nullptr, k, sub, active && sub == 0, {}, {}};
#pragma unroll
  for (int t = 0; t < 4; t++) {
    const int slot = t * S + sub;
    G.sq[t] = slot < 4 ? c_sqr[k][slot] : SqrTerm{-1, -1, 0, 0};
  }
  G.sqh = active ? c_sqr[k][sub >> 1] : SqrTerm{-1, -1, 0, 0};
  Fq2 f = Fq2::one();
  f.c1 = Fq::one();
  f.c0.v[0] += k + blockIdx.x;
  const Fq2 l = f;
  for (int it = 0; it < iters; it++) {
    if constexpr (OP == 0) f = g_sqr<S>(G, f);
    if constexpr (OP == 1) f = g_sqr_h<S>(G, f);
    if constexpr (OP == 3) f = g_mul<S>(G, f, l);
    if constexpr (OP == 4) f = g_line<S>(G, f, l, l, l);
    if constexpr (OP == 5) f = g_line_h<S>(G, f, l, l, l);
    if constexpr (OP == 6) f = g_inv<S>(G, f);
    if constexpr (OP == 7) f = f * l;         // one lane-local Fq2 product (Karatsuba)
    if constexpr (OP == 8) f.c0 = f.c0 * l.c1;  // one Fq product
    if constexpr (OP == 9) f = sub_reduce<S>(f);
    if constexpr (OP == 10) f.c0 = fe_inv(f.c0);
    if constexpr (OP == 11) f.c0 = fq_mul9(f.c0);
    if constexpr (OP == 12) f = f + l;
  }
  if (G.w) out[blockIdx.x * 6 + k] = f;
}

template <int OP>
float run(int blocks, int iters, Fq2* d) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(64), 0, 0, 4, d);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(64), 0, 0, iters, d);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3f / iters;  // us per op
}

int main() {
  Fq2* d;
  hipMalloc(&d, 4096 * 6 * sizeof(Fq2));
  const char* names[] = {"g_sqr", "g_sqr_h", "(unused)", "g_mul", "g_line", "g_line_h", "g_inv",
                         "Fq2 mul (lane)", "Fq mul (lane)", "sub_reduce<8>", "fe_inv", "fq_mul9", "Fq2 add"};
  for (int blocks : {1}) {
    float t[13];
    t[0] = run<0>(blocks, 200, d);
    t[1] = run<1>(blocks, 200, d);
    t[2] = 0.f;
    t[3] = run<3>(blocks, 200, d);
    t[4] = run<4>(blocks, 200, d);
    t[5] = run<5>(blocks, 200, d);
    t[6] = run<6>(blocks, 10, d);
    t[7] = run<7>(blocks, 200, d);
    t[8] = run<8>(blocks, 200, d);
    t[9] = run<9>(blocks, 200, d);
    t[10] = run<10>(blocks, 10, d);
    t[11] = run<11>(blocks, 200, d);
    t[12] = run<12>(blocks, 200, d);
    for (int i = 0; i < 13; i++) printf("blocks=%d %-16s %8.3f us/op\n", blocks, names[i], t[i]);
  }
  return 0;
}
