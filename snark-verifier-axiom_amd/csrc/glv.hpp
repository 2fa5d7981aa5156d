// GLV decomposition for BN254 G1 (device + host).
//
// BN254 G1 has the order-3 endomorphism phi(x, y) = (beta x, y) = [lambda](x, y), so
//   k P = k1 P + k2 phi(P)   with   k = k1 + k2 lambda (mod r),  |k1|, |k2| < 2^127,
// which halves the scalar length of every bucket-method window pass: an n-term MSM becomes a
// 2n-term MSM of 127-bit scalars (W = ceil(128 / c) windows instead of ceil(255 / c)), so the
// number of buckets and the Horner doubling chain both halve while the bucket fill work stays
// 2n * 128 / c = n * 256 / c mixed additions.  This is an implementation choice of the build (the
// reference's Pippenger, snark-verifier/src/util/msm.rs:238-316, uses full-width byte windows);
// the sum it produces is the same group element.
//
// Decomposition (Gallant-Lambert-Vanstone, Babai rounding against the reduced lattice basis
//   v1 = (a1, -B1), v2 = (a2, b2) with a_i + b_i lambda = 0 (mod r), computed by
//   tools/gen_glv.py and checked there):
//   c1 = round(k b2 / r), c2 = round(k B1 / r)   (as floor((k g_i + 2^255) / 2^256), g_i = floor(2^256 x_i / r))
//   k1 = k - c1 a1 - c2 a2,  k2 = c1 B1 - c2 b2
// The rounding error is below 3/4 per coefficient, so |k1| <= 3/4 (a1 + a2) < 2^127 and
// |k2| <= 3/4 (B1 + b2) < 2^127.
#pragma once
#include <cstdint>

#include "field.hpp"

namespace sv {

// beta (Montgomery form, Fq): cube root of unity matching lambda
SV_CONST uint32_t GLV_BETA_MONT[8] = {0xd782e155u, 0x71930c11u, 0xffbe3323u, 0xa6bb947cu,
                                      0xd4741444u, 0xaa303344u, 0x26594943u, 0x2c3b3f0du};
SV_CONST uint32_t GLV_G1[3] = {0xc7e0b3d7u, 0xd91d232eu, 0x00000002u};
SV_CONST uint32_t GLV_G2[5] = {0x391eb18du, 0x7a7bd9d4u, 0xa773d2cfu, 0x4ccef014u, 0x00000002u};
SV_CONST uint32_t GLV_A1[2] = {0x94d213e3u, 0x89d32568u};  // = b2
SV_CONST uint32_t GLV_A2[4] = {0x1221250bu, 0x0be4e154u, 0xeeb859fdu, 0x6f4d8248u};
SV_CONST uint32_t GLV_B1[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u};

// floor((k * g + 2^255) / 2^256) for an NG-limb g: the NG limbs above limb 7
template <int NG>
SV_HD void glv_round_mul(const uint32_t* k, const uint32_t* g, uint32_t* c) {
  uint32_t t[8 + NG];
#pragma unroll
  for (int i = 0; i < 8 + NG; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NG; j++) {
      const uint64_t s = (uint64_t)k[i] * g[j] + t[i + j] + carry;
      t[i + j] = (uint32_t)s;
      carry = s >> 32;
    }
    t[i + NG] = (uint32_t)carry;
  }
  uint64_t s = (uint64_t)t[7] + 0x80000000u;
  uint32_t carry = (uint32_t)(s >> 32);
#pragma unroll
  for (int i = 8; i < 8 + NG; i++) {
    s = (uint64_t)t[i] + carry;
    c[i - 8] = (uint32_t)s;
    carry = (uint32_t)(s >> 32);
  }
}

// p = x * y (mod 2^160), x NX limbs, y NY limbs
template <int NX, int NY>
SV_HD void glv_mul_lo(const uint32_t* x, const uint32_t* y, uint32_t* p) {
#pragma unroll
  for (int i = 0; i < 5; i++) p[i] = 0;
#pragma unroll
  for (int i = 0; i < NX; i++) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < NY; j++) {
      if (i + j < 5) {
        const uint64_t s = (uint64_t)x[i] * y[j] + p[i + j] + carry;
        p[i + j] = (uint32_t)s;
        carry = s >> 32;
      }
    }
    if (i + NY < 5) p[i + NY] = (uint32_t)carry;
  }
}

// acc -= x * y (mod 2^160)
template <int NX, int NY>
SV_HD void glv_sub_mul(uint32_t* acc, const uint32_t* x, const uint32_t* y) {
  uint32_t p[5];
  glv_mul_lo<NX, NY>(x, y, p);
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t s = (uint64_t)acc[i] - p[i] - br;
    acc[i] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
}

// |v| of a 160-bit two's-complement value known to lie in (-2^127, 2^127): 4 magnitude limbs with
// the sign in bit 31 of limb 3
SV_HD void glv_pack(const uint32_t* v, uint32_t* out) {
  const bool neg = (v[4] >> 31) != 0;
  uint64_t c = 1;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    if (neg) {
      c += (uint64_t)(~v[i]);
      out[i] = (uint32_t)c;
      c >>= 32;
    } else {
      out[i] = v[i];
    }
  }
  out[3] |= neg ? 0x80000000u : 0u;
}

// canonical scalar k < r -> (k1, k2) as signed 127-bit halves (glv_pack layout)
SV_HD void glv_split(const uint32_t* k, uint32_t* h1, uint32_t* h2) {
  uint32_t c1[3], c2[5];
  glv_round_mul<3>(k, GLV_G1, c1);
  glv_round_mul<5>(k, GLV_G2, c2);
  uint32_t k1[5] = {k[0], k[1], k[2], k[3], k[4]};
  glv_sub_mul<3, 2>(k1, c1, GLV_A1);
  glv_sub_mul<5, 4>(k1, c2, GLV_A2);
  uint32_t k2[5];
  glv_mul_lo<3, 4>(c1, GLV_B1, k2);    //   c1 B1
  glv_sub_mul<5, 2>(k2, c2, GLV_A1);   // - c2 b2 (b2 = a1)
  glv_pack(k1, h1);
  glv_pack(k2, h2);
}

}  // namespace sv
