// BN254 Fq over 9 x 29-bit limbs (round 4): the bucket accumulation's field.
//
// Why: with 29-bit limbs every partial product is below 2^58, so a Montgomery column of up to 27
// of them (a fused two-product sum) plus the incoming carry stays below 2^63 -- each partial product
// is ONE v_mad_u64_u32 into a 64-bit accumulator, where the 8 x 32-bit product of field.hpp needs a
// v_addc after every v_mad_u64_u32 to keep the carry.  tools/ubench_r29.hip: 172 vs 144 G
// products/s on the MI355X.  Additions pay instead (carries are propagated by shifts), so only the
// product-heavy inner loop (XYZZ mixed additions, curve29.hpp) uses this form; everything it stores
// is converted back to field.hpp's 8 x 32-bit R = 2^256 Montgomery form.
//
// Representation: value * R' mod p with R' = 2^261, little-endian limbs v[0..8], each in
// [0, 2^29) ("normalized"); values are LAZILY reduced -- each operation states the bound of its
// output, always below 2^261.
//   mul / sqr:   inputs below 12p  -> output below 2p   (12^2 p^2 / R' + p < 2p: 144 p < R' = 169.6 p)
//   mul_sum2:    inputs below  9p  -> output below 2p   (2 * 81 p^2 / R' + p < 2p)
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
constexpr uint32_t NP = 0x4866389u;  // -p^-1 mod 2^29

// k p, normalized 29-bit limbs (k = 1, 2, 4, 6)
SV29_HD constexpr uint32_t kp(int k, int i) {
  constexpr uint32_t P1[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                              0x2db40c0u,  0x0a6e141u, 0xe5c2634u,  0x030644eu};
  constexpr uint32_t P2[9] = {0x10f9fa8eu, 0x208c16du, 0x18e5469eu, 0x5aa45a1u, 0xb0bb2f0u,
                              0x5b68181u,  0x14dc282u, 0x1cb84c68u, 0x060c89cu};
  constexpr uint32_t P4[9] = {0x1f3f51cu, 0x41182dbu, 0x11ca8d3cu, 0xb548b43u, 0x161765e0u,
                              0xb6d0302u, 0x29b8504u, 0x197098d0u, 0x0c19139u};
  constexpr uint32_t P6[9] = {0x12edefaau, 0x61a4448u, 0xaafd3dau, 0x10fed0e5u, 0x12318d0u,
                              0x11238484u, 0x3e94786u, 0x1628e538u, 0x12259d6u};
  return k == 1 ? P1[i] : (k == 2 ? P2[i] : (k == 4 ? P4[i] : P6[i]));
}
struct F {
  uint32_t v[L];
};

SV29_HD F zero() {
  F r;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = 0;
  return r;
}
template <int K>
SV29_HD F kp_f() {
  F r;
#pragma unroll
  for (int i = 0; i < L; i++) r.v[i] = kp(K, i);
  return r;
}

// 8 x 32-bit words (a value below 2^256) <-> 9 x 29-bit limbs (the value unchanged)
SV29_HD F from_words(const uint32_t* w) {
  F r;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int bit = 29 * i, j = bit >> 5, s = bit & 31;
    uint32_t x = w[j] >> s;
    if (s > 3 && j + 1 < 8) x |= w[j + 1] << (32 - s);
    r.v[i] = x & MASK;
  }
  return r;
}
SV29_HD void to_words(const F& a, uint32_t* w) {  // a below 2^256
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
      if (i < (k) && j >= 1 && j < L) acc = mad(m[i], kp(1, j), acc);  \
    }                                                                  \
    if ((k) < L) {                                                     \
      m[(k)] = ((uint32_t)acc * NP) & MASK;                            \
      acc = mad(m[(k)], kp(1, 0), acc);                                \
    } else {                                                           \
      t.v[(k) - L] = (uint32_t)acc & MASK;                             \
    }                                                                  \
    acc >>= 29;                                                        \
  }

// a b / R' mod p, below 2p for a, b below 12p
SV29_HD F mul(const F& a, const F& b) {
  uint32_t m[L];
  F t;
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
SV29_HD F sqr(const F& a) {
  uint32_t m[L], a2[L];
  F t;
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
SV29_HD F mul_sum2(const F& a0, const F& b0, const F& a1, const F& b1) {
  uint32_t m[L];
  F t;
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
#undef SV29_REDUCE_COLUMN

// a - b + K p, normalized (b below K p; the result is below bound(a) + K p)
template <int K>
SV29_HD F sub(const F& a, const F& b) {
  F r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)(a.v[i] + kp(K, i)) - (int32_t)b.v[i] + c;
    c = x >> 29;  // arithmetic: floor division by 2^29 (-1, 0 or 1)
    r.v[i] = (uint32_t)x & MASK;
  }
  return r;
}

// a + b, normalized (below bound(a) + bound(b), which must stay below 2^261)
SV29_HD F add(const F& a, const F& b) {
  F r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const uint32_t x = a.v[i] + b.v[i] + c;
    c = x >> 29;
    r.v[i] = x & MASK;
  }
  return r;
}

// a below 2 K p -> below K p: a - K p when that does not go negative
template <int K>
SV29_HD F csub(const F& a) {
  F d;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)kp(K, i) + c;
    c = x >> 29;
    d.v[i] = (uint32_t)x & MASK;
  }
  return c < 0 ? a : d;
}

SV29_HD bool eq(const F& a, const F& b) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < L; i++) x |= a.v[i] ^ b.v[i];
  return x == 0;
}
SV29_HD bool is_zero(const F& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < L; i++) x |= a.v[i];
  return x == 0;
}

// a == 0 mod p for a below 6p: a in {0, p, .., 5p}.  The low limb filters (a match of limb 0 with
// one of the six multiples is needed), so the full comparisons run only on that rare path.
SV29_HD bool is_zero_mod_p_6p(const F& a) {
  constexpr uint32_t LOW[6] = {0u, 0x187cfd47u, 0x10f9fa8eu, 0x976f7d5u, 0x1f3f51cu, 0x1a70f263u};
  bool cand = false;
#pragma unroll
  for (int k = 0; k < 6; k++) cand |= a.v[0] == LOW[k];
  if (!cand) return false;
  // rare: reduce below p by conditional subtractions of 4p, 2p, p (a < 6p < 8p)
  return is_zero(csub<1>(csub<2>(csub<4>(a))));
}

// Form changes without a product: x R' = 32 (x R) mod p, so the way in is a 5-bit shift and a
// small reduction, the way out an exact division by 32 (a Montgomery reduction by 2^5).
// x R (field.hpp's 8 x 32-bit form, below p) -> x R', below 2p
SV29_HD F to_r29(const uint32_t* w) {
  F r;
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
  const uint32_t q = (uint32_t)(((uint64_t)r.v[L - 1] * (0xffffffffull / (kp(1, L - 1) + 1))) >> 32);
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int64_t x = (int64_t)r.v[i] - (int64_t)q * kp(1, i) + c;
    c = x >> 29;
    r.v[i] = (uint32_t)x & MASK;
  }
  return csub<2>(r);
}
// x R' (below 4p) -> x R canonical (below p), as 8 x 32-bit words
SV29_HD void to_r32(const F& a, uint32_t* w) {
  const uint32_t m = (a.v[0] * NP) & 31;  // a + m p = 0 mod 32
  F t;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    c += (uint64_t)m * kp(1, i) + a.v[i];
    t.v[i] = (uint32_t)c & MASK;
    c >>= 29;
  }
  F d;  // (a + m p) / 32, below a / 32 + p < 2p
#pragma unroll
  for (int i = 0; i < L; i++) d.v[i] = (t.v[i] >> 5) | ((i + 1 < L ? t.v[i + 1] : (uint32_t)c) << 24 & MASK);
  to_words(csub<1>(d), w);
}

}  // namespace r29
}  // namespace sv
