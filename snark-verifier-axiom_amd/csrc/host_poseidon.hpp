// Host-side Poseidon transcript over BN254 Fr (4 x 64-bit limbs), for the one serial sponge of
// KzgAs::create_proof (snark-verifier/src/pcs/kzg/accumulation.rs:156-176).
//
// Product code (not the oracle).  create_proof absorbs every accumulator's lhs and rhs into ONE
// fresh PoseidonTranscript (snark-verifier-sdk/src/halo2/aggregation.rs:235-242) and squeezes r:
// 2n field elements -> n + 1 dependent t = 3 permutations, a serial chain of ~260 dependent Fr
// products each.  A GPU lane runs a dependent Fr product in ~0.6 us (one wave), so one
// sponge on the device takes ~20 ms at n = 64; here it takes ~6.4 us per permutation.  The batched
// many-sponge form (one lane per transcript) stays on the device (poseidon.hip).
//
// The schedule is the reference's optimised one (OptimizedPoseidonSpec, poseidon.rs:230-313;
// Poseidon::permutation, :469-500) with the constants of poseidon_consts.hpp (generated from
// oracle/poseidon.py, pinned by the reference KATs poseidon/tests.rs:34-85): folded round
// constants, a pre-sparse MDS after the first full half, sparse partial-round matrices.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

#include "poseidon_consts.hpp"

namespace sv {
namespace host {
namespace fr {

typedef unsigned __int128 u128;

struct E {
  uint64_t l[4];
};

static constexpr uint64_t MOD[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                    0x30644e72e131a029ull};
static constexpr uint64_t NINV = 0xc2e1f593efffffffull;  // -r^-1 mod 2^64
static constexpr uint64_t ONE[4] = {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull,
                                    0x0e0a77c19a07df2full};  // R mod r
static constexpr uint64_t R2[4] = {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull,
                                   0x0216d0b17f4e44a5ull};  // R^2 mod r

inline E one() { return E{{ONE[0], ONE[1], ONE[2], ONE[3]}}; }

// t - r if t >= r (t given as 4 limbs + a carry bit), else t
inline E reduce_once(const uint64_t t[4], uint64_t carry) {
  uint64_t d[4];
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)t[i] - MOD[i] - br;
    d[i] = (uint64_t)s;
    br = (s >> 127) & 1;
  }
  const bool ge = carry || !br;
  E r;
  for (int i = 0; i < 4; i++) r.l[i] = ge ? d[i] : t[i];
  return r;
}

inline E add(const E& a, const E& b) {
  uint64_t t[4];
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    t[i] = (uint64_t)s;
    c = s >> 64;
  }
  return reduce_once(t, (uint64_t)c);
}

inline E mul(const E& a, const E& b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 s = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)s;
      c = s >> 64;
    }
    u128 s = (u128)t[4] + c;
    t[4] = (uint64_t)s;
    t[5] = (uint64_t)(s >> 64);
    const uint64_t m = t[0] * NINV;
    s = (u128)m * MOD[0] + t[0];
    c = s >> 64;
    for (int j = 1; j < 4; j++) {
      s = (u128)m * MOD[j] + t[j] + c;
      t[j - 1] = (uint64_t)s;
      c = s >> 64;
    }
    s = (u128)t[4] + c;
    t[3] = (uint64_t)s;
    t[4] = t[5] + (uint64_t)(s >> 64);
  }
  return reduce_once(t, t[4]);
}

// Lazily reduced product for the permutation: a, b < 2r gives a result below 2r (4 r^2 < 2^256 r),
// no final subtraction.  "No-carry" CIOS: r's top word is below 2^63 - 1, so each row's carries fit
// the N + 1 words (no t[N + 1] word, no extra carry handling).
inline E mul_lazy(const E& a, const E& b) {
  uint64_t t[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a.l[0] * b.l[i] + t[0];
    uint64_t A = (uint64_t)(s >> 64);
    t[0] = (uint64_t)s;
    const uint64_t m = t[0] * NINV;
    s = (u128)m * MOD[0] + t[0];
    uint64_t C = (uint64_t)(s >> 64);
    for (int j = 1; j < 4; j++) {
      s = (u128)a.l[j] * b.l[i] + t[j] + A;
      A = (uint64_t)(s >> 64);
      t[j] = (uint64_t)s;
      s = (u128)m * MOD[j] + t[j] + C;
      C = (uint64_t)(s >> 64);
      t[j - 1] = (uint64_t)s;
    }
    t[3] = C + A;
  }
  return E{{t[0], t[1], t[2], t[3]}};
}

// a + b for a, b < 2r, wrapped below 2r (subtract 2r when the sum reaches it)
inline E add_lazy(const E& a, const E& b) {
  static constexpr uint64_t M2[4] = {0x87c3eb27e0000002ull, 0x5067d090f372e122ull, 0x70a08b6d0302b0baull,
                                     0x60c89ce5c2634053ull};  // 2r
  uint64_t t[4], d[4];
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 x = (u128)a.l[i] + b.l[i] + c;
    t[i] = (uint64_t)x;
    c = x >> 64;
  }
  u128 br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 x = (u128)t[i] - M2[i] - br;
    d[i] = (uint64_t)x;
    br = (x >> 127) & 1;
  }
  const bool ge = c || !br;  // (a + b < 4r < 2^256: c is always 0)
  E r;
  for (int i = 0; i < 4; i++) r.l[i] = ge ? d[i] : t[i];
  return r;
}

// ---- Wide products (round 5): 512-bit unreduced products summed before ONE reduction, so the
// partial rounds' critical path is sqr -> sqr -> (one product + reduction) per round (below).
struct W {  // 512-bit
  uint64_t l[8];
};
inline W mul_wide(const E& a, const E& b) {  // a b, operand scanning (as mul_lazy's rows)
  W r;
  for (int i = 0; i < 8; i++) r.l[i] = 0;
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 s = (u128)a.l[j] * b.l[i] + r.l[i + j] + c;
      r.l[i + j] = (uint64_t)s;
      c = s >> 64;
    }
    r.l[i + 4] = (uint64_t)c;
  }
  return r;
}
inline W add_wide(const W& a, const W& b) {
  W r;
  u128 c = 0;
  for (int i = 0; i < 8; i++) {
    const u128 s = (u128)a.l[i] + b.l[i] + c;
    r.l[i] = (uint64_t)s;
    c = s >> 64;
  }
  return r;
}
// T / 2^256 mod r for T < 2^256 r + ... : (T + m r) / 2^256 < T / 2^256 + r; wrapped below 2r
// (one conditional subtraction of 2r) when that is below 4r, i.e. for T < 3 * 2^256 r
inline E redc_wide(const W& T) {
  uint64_t t[8];
  for (int i = 0; i < 8; i++) t[i] = T.l[i];
  for (int i = 0; i < 4; i++) {  // T + m r < 2^512 for the bounds above: no carry out of t[7]
    const uint64_t m = t[i] * NINV;
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 s = (u128)m * MOD[j] + t[i + j] + c;
      t[i + j] = (uint64_t)s;
      c = s >> 64;
    }
    for (int j = i + 4; j < 8; j++) {
      const u128 s = (u128)t[j] + c;
      t[j] = (uint64_t)s;
      c = s >> 64;
    }
  }
  return add_lazy(E{{t[4], t[5], t[6], t[7]}}, E{{0, 0, 0, 0}});
}
inline E sqr_lazy(const E& a) { return mul_lazy(a, a); }

inline E to_mont(const E& a) { return mul(a, E{{R2[0], R2[1], R2[2], R2[3]}}); }
inline E from_mont(const E& a) { return mul(a, E{{1, 0, 0, 0}}); }

// a canonical integer below 2r (e.g. an Fq coordinate: p < 2r) reduced mod r: fe_to_fe
// (util/arithmetic.rs:256-258) of a base-field element
inline E reduce_below_2r(const E& a) { return reduce_once(a.l, 0); }

inline bool is_reduced(const E& a) {
  for (int i = 3; i >= 0; i--) {
    if (a.l[i] < MOD[i]) return true;
    if (a.l[i] > MOD[i]) return false;
  }
  return false;
}

// the t = 3 constants of poseidon_consts.hpp (8 x u32 Montgomery limbs each) as 4 x u64
struct Spec3 {
  static constexpr int T = 3, RF = SV_POSEIDON_T3_RF, RP = SV_POSEIDON_T3_RP;
  std::vector<E> start, partial, end, mds, pre, sparse;
  static std::vector<E> load(const uint32_t* w, size_t words) {
    std::vector<E> v(words / 8);
    for (size_t i = 0; i < v.size(); i++)
      for (int k = 0; k < 4; k++) v[i].l[k] = (uint64_t)w[8 * i + 2 * k] | ((uint64_t)w[8 * i + 2 * k + 1] << 32);
    return v;
  }
  Spec3() {
    static const uint32_t c_start[] = SV_POSEIDON_T3_START_INIT, c_partial[] = SV_POSEIDON_T3_PARTIAL_INIT,
                          c_end[] = SV_POSEIDON_T3_END_INIT, c_mds[] = SV_POSEIDON_T3_MDS_INIT,
                          c_pre[] = SV_POSEIDON_T3_PRE_INIT, c_sparse[] = SV_POSEIDON_T3_SPARSE_INIT;
    start = load(c_start, sizeof(c_start) / 4);
    partial = load(c_partial, sizeof(c_partial) / 4);
    end = load(c_end, sizeof(c_end) / 4);
    mds = load(c_mds, sizeof(c_mds) / 4);
    pre = load(c_pre, sizeof(c_pre) / 4);
    sparse = load(c_sparse, sizeof(c_sparse) / 4);
  }
  static const Spec3& get() {
    static const Spec3 s;
    return s;
  }
};

// One full round in the plain order: s_j <- s_j^5 + c_j (c = nullptr: none), then each MDS row as
// ONE reduction of three wide products (below 3 (2r) r = 6 r^2 < 3 * 2^256 r).
inline void full_round3p(E (&s)[3], const E* m, const E* c) {
  E x[3];
  for (int j = 0; j < 3; j++) {
    const E x2 = sqr_lazy(s[j]);
    x[j] = mul_lazy(sqr_lazy(x2), s[j]);
    if (c) x[j] = add_lazy(x[j], c[j]);
  }
  for (int i = 0; i < 3; i++)
    s[i] = redc_wide(add_wide(mul_wide(x[0], m[3 * i]), add_wide(mul_wide(x[1], m[3 * i + 1]), mul_wide(x[2], m[3 * i + 2]))));
}

// Poseidon::permutation (poseidon.rs:469-500) after the inputs were added: the bare HADES map in
// the optimised schedule, as the device's sv::permute<3> runs it (Montgomery form).  Every word
// stays below 2r inside (lazy products and sums); the state is canonical again at the end.
// Round 5: a partial round forms row1 s1 + row2 s2 (two wide products) beside the pow5 chain and
// reduces the row once with (s0^5 + c) row0 added: the same products as before, the chain shorter
// by the row's other two products (6.72 -> 6.40 us per permutation on the box's EPYC 9575F,
// tools/ubench_host_poseidon.cpp; folding the constants to shorten it further did more work and
// measured 7.6 us: the host chain is bound by multiplier throughput as much as by latency).
inline void permute3(E (&s)[3]) {
  const Spec3& sp = Spec3::get();
  constexpr int H = Spec3::RF / 2;
  for (int i = 0; i < 3; i++) s[i] = add_lazy(s[i], sp.start[i]);  // absorb_with_pre_constants
  for (int r = 1; r <= H; r++) full_round3p(s, r < H ? sp.mds.data() : sp.pre.data(), &sp.start[r * 3]);
  for (int r = 0; r < Spec3::RP; r++) {
    const E* row = sp.sparse.data() + r * 5;  // row (3) || col_hat (2)
    const E x = s[0];
    const W u = add_wide(mul_wide(s[1], row[1]), mul_wide(s[2], row[2]));  // beside the pow5 chain
    const E x2 = sqr_lazy(x);
    const E x5c = add_lazy(mul_lazy(sqr_lazy(x2), x), sp.partial[r]);
    s[0] = redc_wide(add_wide(u, mul_wide(x5c, row[0])));
    for (int i = 1; i < 3; i++) s[i] = add_lazy(s[i], mul_lazy(x5c, row[3 + i - 1]));
  }
  for (int r = 0; r < H; r++) full_round3p(s, sp.mds.data(), r < H - 1 ? &sp.end[r * 3] : nullptr);
  for (int i = 0; i < 3; i++) s[i] = reduce_once(s[i].l, 0);  // [0, 2r) -> canonical
}

// Poseidon<Fr, Fr, 3, 2> with the NativeLoader (poseidon.rs:412-467): update buffers, squeeze
// absorbs RATE = 2 elements per permutation (a short last chunk padded with a single 1) and runs
// one more permutation on the padded empty chunk when the buffer length is a multiple of RATE.
struct Sponge3 {
  E st[3];
  std::vector<E> buf;
  Sponge3() {
    // State::default (poseidon.rs:335-342): capacity element 2^64
    st[0] = to_mont(E{{0, 1, 0, 0}});
    st[1] = st[2] = E{{0, 0, 0, 0}};
  }
  void update(const E& m) { buf.push_back(m); }
  E squeeze() {
    const size_t n = buf.size();
    for (size_t p = 0; p < n; p += 2) {
      const size_t m = n - p < 2 ? n - p : 2;
      for (size_t k = 0; k < m; k++) st[1 + k] = add(st[1 + k], buf[p + k]);
      if (m < 2) st[1 + m] = add(st[1 + m], one());
      permute3(st);
    }
    if (n % 2 == 0) {
      st[1] = add(st[1], one());
      permute3(st);
    }
    buf.clear();
    return st[1];
  }
};

}  // namespace fr
}  // namespace host
}  // namespace sv
