// BN254 Fq and Fr over 9 x 29-bit limbs (round 4): the bucket accumulation's field (Fq) and the
// Poseidon permutation's (Fr).
//
// Why: with 29-bit limbs every partial product is below 2^58, so a Montgomery column of up to 27
// of them (a fused two-product sum) plus the incoming carry stays below 2^63 -- each partial product
// is ONE v_mad_u64_u32 into a 64-bit accumulator, where the 8 x 32-bit product of field.hpp needs a
// v_addc after every v_mad_u64_u32 to keep the carry.  tools/ubench_r29.hip: 172 vs 144 G
// products/s on the MI355X.  Additions pay instead (carries are propagated by shifts), so only the
// product-heavy loops use this form (the XYZZ mixed additions of curve29.hpp, the Poseidon rounds);
// what leaves them is converted back to field.hpp's 8 x 32-bit R = 2^256 Montgomery form.  The
// modulus is a type parameter (FqM29 = p, FrM29 = r; F29<M> carries it); F = F29<FqM29>.
//
// Representation (p below stands for the modulus; both are below 2^254 and above 2^253):
// value * R' mod p with R' = 2^261, little-endian limbs v[0..8], each in
// [0, 2^29) ("normalized"); values are LAZILY reduced -- each operation states the bound of its
// output, always below 2^261.
//   mul / sqr:   inputs below 12p  -> output below 2p   (12^2 p^2 / R' + p < 2p: 144 p < R' = 169.6 p)
//   mul_sum2:    inputs below  9p  -> output below 2p   (2 * 81 p^2 / R' + p < 2p)
//   mul_sum3:    a_i below 9p, b_i below p -> output below 2p (3 * 9 p^2 / R' + p < 2p; a column
//                holds 27 + 9 partial products below 2^58 and the carry: below 2^64)
//   sub<K>:      a - b + K p for b below K p -> below (bound of a) + K p
//   csub<K>:     a below 2 K p -> below K p (one conditional subtraction of K p)
// Host build: the same code runs on the CPU (tests/native/field29check.cpp checks every operation
// and bound against Python big integers).
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define SV29_HD __host__ __device__ __forceinline__
#else
#define SV29_HD inline
#endif

namespace sv {
namespace r29 {

constexpr int L = 9;
constexpr uint32_t MASK = (1u << 29) - 1;

// the moduli: k * modulus as normalized 29-bit limbs (k = 0..8) and -modulus^-1 mod 2^29
struct FqM29 {  // p
  static constexpr uint32_t NP = 0x4866389u;
  SV29_HD static constexpr uint32_t kp(int k, int i) {
    constexpr uint32_t T[9][9] = {
        {0, 0, 0, 0, 0, 0, 0, 0, 0},
        {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u, 0x2db40c0u, 0xa6e141u, 0xe5c2634u, 0x30644eu},
        {0x10f9fa8eu, 0x208c16du, 0x18e5469eu, 0x5aa45a1u, 0xb0bb2f0u, 0x5b68181u, 0x14dc282u, 0x1cb84c68u, 0x60c89cu},
        {0x976f7d5u, 0x30d2224u, 0x1557e9edu, 0x87f6872u, 0x918c68u, 0x891c242u, 0x1f4a3c3u, 0xb14729cu, 0x912cebu},
        {0x1f3f51cu, 0x41182dbu, 0x11ca8d3cu, 0xb548b43u, 0x161765e0u, 0xb6d0302u, 0x29b8504u, 0x197098d0u, 0xc19139u},
        {0x1a70f263u, 0x515e391u, 0xe3d308bu, 0xe29ae14u, 0xb9d3f58u, 0xe4843c3u, 0x3426645u, 0x7ccbf04u, 0xf1f588u},
        {0x12edefaau, 0x61a4448u, 0xaafd3dau, 0x10fed0e5u, 0x12318d0u, 0x11238484u, 0x3e94786u, 0x1628e538u, 0x12259d6u},
        {0xb6aecf1u, 0x71ea4ffu, 0x7227729u, 0x13d3f3b6u, 0x16a8f248u, 0x13fec544u, 0x49028c7u, 0x4850b6cu, 0x152be25u},
        {0x3e7ea38u, 0x82305b6u, 0x3951a78u, 0x16a91687u, 0xc2ecbc0u, 0x16da0605u, 0x5370a08u, 0x12e131a0u, 0x1832273u}};
    return T[k][i];
  }
};
struct FrM29 {  // r
  static constexpr uint32_t NP = 0xfffffffu;
  SV29_HD static constexpr uint32_t kp(int k, int i) {
    constexpr uint32_t T[9][9] = {
        {0, 0, 0, 0, 0, 0, 0, 0, 0},
        {0x10000001u, 0x1f0fac9fu, 0xe5c2450u, 0x7d090f3u, 0x1585d283u, 0x2db40c0u, 0xa6e141u, 0xe5c2634u, 0x30644eu},
        {0x2u, 0x1e1f593fu, 0x1cb848a1u, 0xfa121e6u, 0xb0ba506u, 0x5b68181u, 0x14dc282u, 0x1cb84c68u, 0x60c89cu},
        {0x10000003u, 0x1d2f05deu, 0xb146cf2u, 0x1771b2dau, 0x917789u, 0x891c242u, 0x1f4a3c3u, 0xb14729cu, 0x912cebu},
        {0x4u, 0x1c3eb27eu, 0x19709143u, 0x1f4243cdu, 0x16174a0cu, 0xb6d0302u, 0x29b8504u, 0x197098d0u, 0xc19139u},
        {0x10000005u, 0x1b4e5f1du, 0x7ccb594u, 0x712d4c1u, 0xb9d1c90u, 0xe4843c3u, 0x3426645u, 0x7ccbf04u, 0xf1f588u},
        {0x6u, 0x1a5e0bbdu, 0x1628d9e5u, 0xee365b4u, 0x122ef13u, 0x11238484u, 0x3e94786u, 0x1628e538u, 0x12259d6u},
        {0x10000007u, 0x196db85cu, 0x484fe36u, 0x16b3f6a8u, 0x16a8c196u, 0x13fec544u, 0x49028c7u, 0x4850b6cu, 0x152be25u},
        {0x8u, 0x187d64fcu, 0x12e12287u, 0x1e84879bu, 0xc2e9419u, 0x16da0605u, 0x5370a08u, 0x12e131a0u, 0x1832273u}};
    return T[k][i];
  }
};

template <class M>
struct F29 {
  uint32_t v[L];
};
using F = F29<FqM29>;

template <class M = FqM29>
SV29_HD F29<M> zero() {
  F29<M> r;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = 0;
  return r;
}
template <int K, class M = FqM29>
SV29_HD F29<M> kp_f() {
  F29<M> r;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = M::kp(K, i);
  return r;
}

// 8 x 32-bit words (a value below 2^256) <-> 9 x 29-bit limbs (the value unchanged)
template <class M = FqM29>
SV29_HD F29<M> from_words(const uint32_t* w) {
  F29<M> r;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int bit = 29 * i, j = bit >> 5, s = bit & 31;
    uint32_t x = w[j] >> s;
    if (s > 3 && j + 1 < 8) x |= w[j + 1] << (32 - s);
    r.v[i] = x & MASK;
  }
  return r;
}
template <class M>
SV29_HD void to_words(const F29<M>& a, uint32_t* w) {  // a below 2^256
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int bit = 32 * j, i = bit / 29, s = bit % 29;
    uint32_t x = a.v[i] >> s;
    if (i + 1 < L) x |= a.v[i + 1] << (29 - s);
    if (s > 26 && i + 2 < L) x |= a.v[i + 2] << (58 - s);
    w[j] = x;
  }
}

SV29_HD uint64_t mad(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }  // v_mad_u64_u32

// Montgomery reduction tail shared by the products: column k's sum in acc (products of the inputs
// already added), m_i p_{k-i} for i < k added here; the low 9 columns fix m_k, the high ones give t.
#define SV29_REDUCE_COLUMN(k)                                          \
  {                                                                    \
    _Pragma("unroll") for (int i = 0; i < L; i++) {                    \
      const int j = (k) - i;                                           \
      if (i < (k) && j >= 1 && j < L) acc = mad(m[i], M::kp(1, j), acc); \
    }                                                                  \
    if ((k) < L) {                                                     \
      m[(k)] = ((uint32_t)acc * M::NP) & MASK;                         \
      acc = mad(m[(k)], M::kp(1, 0), acc);                             \
    } else {                                                           \
      t.v[(k) - L] = (uint32_t)acc & MASK;                             \
    }                                                                  \
    acc >>= 29;                                                        \
  }

// a b / R' mod p, below 2p for a, b below 12p
template <class M>
SV29_HD F29<M> mul(const F29<M>& a, const F29<M>& b) {
  uint32_t m[L];
  F29<M> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) acc = mad(a.v[i], b.v[j], acc);
    }
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

// a^2 / R' mod p, below 2p for a below 12p: the cross products once, against 2 a_j
template <class M>
SV29_HD F29<M> sqr(const F29<M>& a) {
  uint32_t m[L], a2[L];
  F29<M> t;
#pragma unroll
  for (int i = 0; i < L; i++) a2[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j > i && j < L) acc = mad(a.v[i], a2[j], acc);
    }
    if ((k & 1) == 0 && k / 2 < L) acc = mad(a.v[k / 2], a.v[k / 2], acc);
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

// (a0 b0 + a1 b1) / R' mod p with ONE reduction, below 2p for inputs below 9p (a column: at most
// 27 products below 2^58 plus the carry, below 2^63)
template <class M>
SV29_HD F29<M> mul_sum2(const F29<M>& a0, const F29<M>& b0, const F29<M>& a1, const F29<M>& b1) {
  uint32_t m[L];
  F29<M> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) {
        acc = mad(a0.v[i], b0.v[j], acc);
        acc = mad(a1.v[i], b1.v[j], acc);
      }
    }
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}
// (a0 b0 + a1 b1 + a2 b2) / R' mod p with ONE reduction, below 2p for a_i below 9p and b_i below p
// (an MDS row over constants)
template <class M>
SV29_HD F29<M> mul_sum3(const F29<M>& a0, const F29<M>& b0, const F29<M>& a1, const F29<M>& b1,
                        const F29<M>& a2, const F29<M>& b2) {
  uint32_t m[L];
  F29<M> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) {
        acc = mad(a0.v[i], b0.v[j], acc);
        acc = mad(a1.v[i], b1.v[j], acc);
        acc = mad(a2.v[i], b2.v[j], acc);
      }
    }
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}
// Round 6: a product with a normalized subtraction fused into its high columns.  The caller's
// per-limb addends D_i (each in [0, 2^32)) go into column L + i before the column's carry-out, so
// the result is a b / R' + sum D_i 2^(29 i), with the top limb masked to 29 bits: multiples of 2^261
// vanish.  A subtraction a b / R' + K p - c becomes D_i = K p_i + 2^29 - [i > 0] - c_i (the
// borrow of 2^29 per limb sums to exactly 2^261), which saves the separate pass's per-limb add,
// arithmetic shift and mask.  The caller guarantees that the true value lies in [0, 2^261).
template <class M>
SV29_HD F29<M> mul_add_hi(const F29<M>& a, const F29<M>& b, const uint32_t D[L]) {
  uint32_t m[L];
  F29<M> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
    if (k >= L) acc += D[k - L];
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) acc = mad(a.v[i], b.v[j], acc);
    }
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = ((uint32_t)acc + D[L - 1]) & MASK;
  return t;
}
template <class M>
SV29_HD F29<M> sqr_add_hi(const F29<M>& a, const uint32_t D[L]) {
  uint32_t m[L], a2[L];
  F29<M> t;
#pragma unroll
  for (int i = 0; i < L; i++) a2[i] = a.v[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
    if (k >= L) acc += D[k - L];
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j > i && j < L) acc = mad(a.v[i], a2[j], acc);
    }
    if ((k & 1) == 0 && k / 2 < L) acc = mad(a.v[k / 2], a.v[k / 2], acc);
    SV29_REDUCE_COLUMN(k)
  }
  t.v[L - 1] = ((uint32_t)acc + D[L - 1]) & MASK;
  return t;
}
#undef SV29_REDUCE_COLUMN

// a b / R' + K p - c (c normalized, below K p; the result below 2p + K p): mul_add_hi
template <int K, class M>
SV29_HD F29<M> mul_sub(const F29<M>& a, const F29<M>& b, const F29<M>& c) {
  uint32_t D[L];
#pragma unroll
  for (int i = 0; i < L; i++) D[i] = (M::kp(K, i) + (1u << 29) - (i > 0 ? 1u : 0u)) - c.v[i];
  return mul_add_hi(a, b, D);
}
// a^2 / R' + K p - b - 2 c (b, c normalized, b + 2c below K p; below 2p + K p): the XYZZ
// addition's X3 = R^2 - PPP - 2Q + 6p in the square's high columns
template <int K, class M>
SV29_HD F29<M> sqr_sub2c(const F29<M>& a, const F29<M>& b, const F29<M>& c) {
  uint32_t D[L];
#pragma unroll
  for (int i = 0; i < L; i++) D[i] = (M::kp(K, i) + (3u << 29) - (i > 0 ? 3u : 0u)) - (b.v[i] + (c.v[i] << 1));
  return sqr_add_hi(a, D);
}

// a b / R' mod p like mul (inputs below 12p -> output below 2p), scheduled for the latency of ONE
// wave (the decider's lane products, round 5): the 81 partial products go to 17 separate 64-bit
// column accumulators (consecutive mads are independent), then 9 reduction steps, each a short
// dependent chain (m from the column's low word, the m p_0 mad, the carry into the next column)
// with its 8 other mads off the chain.  A column collects at most 9 + 9 products below 2^58 plus a
// carry below 2^35: below 2^63.
template <class M>
SV29_HD F29<M> mul_ilp(const F29<M>& a, const F29<M>& b) {
  uint64_t c[2 * L - 1];
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) c[k] = 0;
#pragma unroll
  for (int i = 0; i < L; i++)
#pragma unroll
    for (int j = 0; j < L; j++) c[i + j] = mad(a.v[i], b.v[j], c[i + j]);
#pragma unroll
  for (int k = 0; k < L; k++) {
    const uint32_t m = ((uint32_t)c[k] * M::NP) & MASK;
    c[k] = mad(m, M::kp(1, 0), c[k]);  // the low 29 bits are now zero
    c[k + 1] += c[k] >> 29;
#pragma unroll
    for (int j = 1; j < L; j++) c[k + j] = mad(m, M::kp(1, j), c[k + j]);
  }
  F29<M> t;
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < L - 1; i++) {
    const uint64_t x = c[L + i] + carry;
    t.v[i] = (uint32_t)x & MASK;
    carry = x >> 29;
  }
  t.v[L - 1] = (uint32_t)carry;
  return t;
}

// a - b + K p, normalized (b below K p; the result is below bound(a) + K p)
template <int K, class M>
SV29_HD F29<M> sub(const F29<M>& a, const F29<M>& b) {
  F29<M> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)(a.v[i] + M::kp(K, i)) - (int32_t)b.v[i] + c;
    c = x >> 29;  // arithmetic: floor division by 2^29 (-1, 0 or 1)
    r.v[i] = (uint32_t)x & MASK;
  }
  return r;
}

// a + b, normalized (below bound(a) + bound(b), which must stay below 2^261)
template <class M>
SV29_HD F29<M> add(const F29<M>& a, const F29<M>& b) {
  F29<M> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const uint32_t x = a.v[i] + b.v[i] + c;
    c = x >> 29;
    r.v[i] = x & MASK;
  }
  return r;
}

// a + K p - b - 2 c in ONE normalized pass (round 5: the XYZZ addition's X3 = R^2 - PPP - 2Q + 6p
// without its three passes and the conditional subtraction), for normalized b, c and a value in
// [0, 2^261); a limb's partial sum stays inside int32 (above -3 * 2^29 - 4, below 2^30 + 2)
template <int K, class M>
SV29_HD F29<M> sub_2c(const F29<M>& a, const F29<M>& b, const F29<M>& c) {
  F29<M> r;
  int32_t cy = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)(a.v[i] + M::kp(K, i)) - (int32_t)b.v[i] - 2 * (int32_t)c.v[i] + cy;
    cy = x >> 29;  // arithmetic: floor division by 2^29 (-3 .. 1)
    r.v[i] = (uint32_t)x & MASK;
  }
  return r;
}

// (neg ? -a : a) + K p - b in one normalized pass (round 5: the bucket chain's Rd = +-S2 - Y + 4p,
// the point's sign applied to S2 instead of negating y2 for every entry), for normalized a, b and a
// value in [0, 2^261); a limb's partial sum stays inside int32
template <int K, class M>
SV29_HD F29<M> sub_sgn(const F29<M>& a, bool neg, const F29<M>& b) {
  F29<M> r;
  int32_t cy = 0;
  const uint32_t sgn = neg ? 0xffffffffu : 1u;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)(a.v[i] * sgn) + (int32_t)M::kp(K, i) - (int32_t)b.v[i] + cy;
    cy = x >> 29;  // arithmetic: floor division by 2^29 (-2 .. 1)
    r.v[i] = (uint32_t)x & MASK;
  }
  return r;
}

// a below 2 K p -> below K p: a - K p when that does not go negative
template <int K, class M>
SV29_HD F29<M> csub(const F29<M>& a) {
  F29<M> d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)M::kp(K, i) + c;
    c = x >> 29;
    d.v[i] = (uint32_t)x & MASK;
  }
  return c < 0 ? a : d;
}

template <class M>
SV29_HD bool eq(const F29<M>& a, const F29<M>& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < L; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}
template <class M>
SV29_HD bool is_zero(const F29<M>& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < L; i++) x |= a.v[i];
  return x == 0;
}

// a == 0 mod p for a below 16p (Fq only): a in {0, p, .., 15p}.  Round 6: the one multiple k p a
// can equal comes from its top limb, k = round(a_8 / (p / 2^232)) in float (the multiples' top
// limbs are ~3.17e6 apart, so the rounding is exact for every k < 16; tests/test_field29.py checks
// all sixteen), and limb 0 must match k p's; the full comparison runs only on that rare path.  The
// round-5 filter compared limb 0 with each multiple, which the compiler lowered to a binary search
// of divergent branches: ~60 SALU instructions per bucket entry.
SV29_HD bool is_zero_mod_p_16p(const F& a) {
  constexpr float kInvPTop = 3.1531752142655023e-07f;  // 2^232 / p
  const uint32_t k = (uint32_t)((float)a.v[L - 1] * kInvPTop + 0.5f);
  if (a.v[0] != ((k * FqM29::kp(1, 0)) & MASK)) return false;
  // rare: reduce below p by conditional subtractions of 8p, 4p, 2p, p
  return is_zero(csub<1>(csub<2>(csub<4>(csub<8>(a)))));
}
SV29_HD bool is_zero_mod_p_6p(const F& a) { return is_zero_mod_p_16p(a); }
// (round 5: the bucket chain's Pd = U2 - X + 8p with X below 8p is below 10p)
SV29_HD bool is_zero_mod_p_10p(const F& a) { return is_zero_mod_p_16p(a); }

// Form changes without a product: x R' = 32 (x R) mod p, so the way in is a 5-bit shift and a
// small reduction, the way out an exact division by 32 (a Montgomery reduction by 2^5).
// x R (field.hpp's 8 x 32-bit form, below p) -> x R', below 2p
template <class M = FqM29>
SV29_HD F29<M> to_r29(const uint32_t* w) {
  F29<M> r;
#pragma unroll
  for (int i = 0; i < L; i++) {  // limb i = bits [29 i - 5, 29 i + 24) of the value
    if (i == 0) {
      r.v[0] = (w[0] << 5) & MASK;
      continue;
    }
    const int bit = 29 * i - 5, j = bit >> 5, s = bit & 31;
    uint32_t x = w[j] >> s;
    if (s > 3 && j + 1 < 8) x |= w[j + 1] << (32 - s);
    r.v[i] = x & MASK;
  }
  // r = 32 x R < 32 p: subtract q p, q = floor(r8 / (p8 + 1)) from the top limbs (a multiply-high
  // by floor(2^32 / (p8 + 1))); q is at most 2 below floor(r / p), so the rest is below 3p
  const uint32_t q = (uint32_t)(((uint64_t)r.v[L - 1] * (0xffffffffull / (M::kp(1, L - 1) + 1))) >> 32);
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int64_t x = (int64_t)r.v[i] - (int64_t)q * M::kp(1, i) + c;
    c = x >> 29;
    r.v[i] = (uint32_t)x & MASK;
  }
  return csub<2>(r);
}
// x R' (below 4p) -> x R canonical (below p), as 8 x 32-bit words
template <class M>
SV29_HD void to_r32(const F29<M>& a, uint32_t* w) {
  const uint32_t m = (a.v[0] * M::NP) & 31;  // a + m p = 0 mod 32
  F29<M> t;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    c += (uint64_t)m * M::kp(1, i) + a.v[i];
    t.v[i] = (uint32_t)c & MASK;
    c >>= 29;
  }
  F29<M> d;  // (a + m p) / 32, below a / 32 + p < 2p
#pragma unroll
  for (int i = 0; i < L; i++) d.v[i] = (t.v[i] >> 5) | ((i + 1 < L ? t.v[i + 1] : (uint32_t)c) << 24 & MASK);
  to_words(csub<1>(d), w);
}

}  // namespace r29
}  // namespace sv
