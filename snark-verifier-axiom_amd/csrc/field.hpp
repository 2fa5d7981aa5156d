// BN254 field arithmetic for gfx950 (and the host, for the same templates' unit checks).
//
// Fq / Fr are 8 x 32-bit little-endian limbs in Montgomery form with R = 2^256 -- byte-for-byte
// the halo2curves in-memory layout (4 x u64 LE Montgomery), so device buffers can be filled
// from halo2curves memory with no conversion.  Replaces the halo2curves 0.3.1 Fq/Fr ops that
// snark-verifier's hot path bottoms out in (reached via snark-verifier/src/util/arithmetic.rs:5-13).
//
// Montgomery multiplication on the device is finely-integrated product scanning over 32-bit limbs:
// every partial product is one v_mad_u64_u32 (32x32+64 -> 64, ~30 per clock per CU, measured
// 18.2 T/s chip-wide by tools/ubench_fpmul.hip) whose carry-out feeds a v_addc -- 128 products,
// 130 G mul/s (round-1 variable-operand microbenchmark; its binary was dropped from the tree).  The host build of the same templates uses portable CIOS.
// Elements are kept fully reduced in [0, p) so equality is bitwise.
#pragma once
#include <cstdint>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define SV_HD __host__ __device__ __forceinline__
#define SV_NOINL __host__ __device__ inline __attribute__((noinline))
#else
#define SV_HD inline
#define SV_NOINL inline
#endif

#include "bn254_consts.hpp"

namespace sv {

struct FqTag {
  SV_HD static uint32_t p(int i) { return FQ_P[i]; }
  SV_HD static uint32_t one(int i) { return FQ_ONE[i]; }
  SV_HD static uint32_t r2(int i) { return FQ_R2[i]; }
  static constexpr uint32_t NP0 = FQ_NP0;
};
struct FrTag {
  SV_HD static uint32_t p(int i) { return FR_P[i]; }
  SV_HD static uint32_t one(int i) { return FR_ONE[i]; }
  SV_HD static uint32_t r2(int i) { return FR_R2[i]; }
  static constexpr uint32_t NP0 = FR_NP0;
};

template <class M>
struct Fe {
  uint32_t v[8];

  SV_HD static Fe zero() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  SV_HD static Fe one() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = M::one(i);
    return r;
  }
  SV_HD static Fe modulus() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = M::p(i);
    return r;
  }
  SV_HD bool is_zero() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i];
    return acc == 0;
  }
  SV_HD bool operator==(const Fe& o) const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i] ^ o.v[i];
    return acc == 0;
  }
  SV_HD bool operator!=(const Fe& o) const { return !(*this == o); }
  // true when the raw limbs are < modulus
  SV_HD bool is_reduced() const {
    uint64_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t s = (uint64_t)v[i] - M::p(i) - br;
      br = (s >> 63) & 1;
    }
    return br == 1;
  }
};

template <class M>
SV_HD Fe<M> fe_select(bool c, const Fe<M>& a, const Fe<M>& b) {
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Device add/sub as explicit carry chains (__builtin_addc/subc -> v_addc/v_subb through an SGPR pair,
// 32 VALU per op instead of ~90 for the 64-bit-intermediate C form).  A VALU carry-out read by the
// next v_addc needs two wait states, so a lone chain issues one useful instruction per three slots;
// the loops below are fused so the compiler interleaves independent chains (the trial subtraction
// of p lags the addition by one limb) and the wait states fill with useful work -- this matters
// for the single-wave latency-bound code (decider, Horner chains, tails).
template <class M>
SV_HD Fe<M> operator+(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> t, d, r;
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    // a + b < 2p < 2^255: no carry out; subtract p when t >= p
    d.v[i] = __builtin_subc(t.v[i], M::p(i), br, &br);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = br ? t.v[i] : d.v[i];
  return r;
}

template <class M>
SV_HD Fe<M> operator-(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> t, r;
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;  // add p back on borrow
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __builtin_addc(t.v[i], M::p(i) & mask, c, &c);
  return r;
}

// Latency form of a - b for chains that run on a single wave: a - b and a + (p - b) as three
// independent carry chains (no wait for the final borrow before the correction), then a select.
template <class M>
SV_HD Fe<M> fe_sub_lat(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> t, w, u, r;
  uint32_t b1 = 0, b2 = 0, c3 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t.v[i] = __builtin_subc(a.v[i], b.v[i], b1, &b1);
    w.v[i] = __builtin_subc(M::p(i), b.v[i], b2, &b2);
    u.v[i] = __builtin_addc(a.v[i], w.v[i], c3, &c3);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = b1 ? u.v[i] : t.v[i];
  return r;
}
#else
template <class M>
SV_HD Fe<M> operator+(const Fe<M>& a, const Fe<M>& b) {
  uint32_t t[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[i] + b.v[i] + c;
    t[i] = (uint32_t)s;
    c = s >> 32;
  }
  // a + b < 2p < 2^255: no carry out; subtract p when t >= p
  Fe<M> d;
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)t[i] - M::p(i) - br;
    d.v[i] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  Fe<M> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = br ? t[i] : d.v[i];
  return r;
}

template <class M>
SV_HD Fe<M> operator-(const Fe<M>& a, const Fe<M>& b) {
  uint32_t t[8];
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a.v[i] - b.v[i] - br;
    t[i] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  uint32_t mask = 0u - (uint32_t)br;  // add p back on borrow
  Fe<M> r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)t[i] + (M::p(i) & mask) + c;
    r.v[i] = (uint32_t)s;
    c = s >> 32;
  }
  return r;
}

template <class M>
SV_HD Fe<M> fe_sub_lat(const Fe<M>& a, const Fe<M>& b) {
  return a - b;
}
#endif

template <class M>
SV_HD Fe<M> operator-(const Fe<M>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  // p - a with one borrow chain; -0 = 0
  Fe<M> r;
  uint32_t br = 0, nz = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i] = __builtin_subc(M::p(i), a.v[i], br, &br);
    nz |= a.v[i];
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = nz ? r.v[i] : 0u;
  return r;
#else
  return Fe<M>::zero() - a;
#endif
}

template <class M>
SV_HD Fe<M> fe_dbl(const Fe<M>& a) {
  return a + a;
}

#if defined(__HIP_DEVICE_COMPILE__)
// acc (64 bit) += a * b with the carry out of v_mad_u64_u32 collected in ovf: two VALU
// instructions per partial product and no re-packing of 64-bit addends (the compiler's CIOS
// lowering spends ~2.3 v_mov per product on that; round-1 microbenchmark: 99.6 -> 130 G mul/s).
// VCC hazard: the v_addc reads VCC right after the quarter-rate v_mad_u64_u32 wrote it; the mad's
// multi-pass issue occupies the wave's VALU past the 2-state VALU-SGPR-write window, so no s_nop is
// needed inside a block (every result is checked bit-exact against the oracle in tests/).  hipcc
// pads one state after each asm block, so products are issued four per block (single-wave latency
// 737 -> 607 ns per multiply, round-1 microbenchmark; tools/ubench_wg.hip measures the
// current per-product latency: 1517 cycles per dependent product on one wave).
#define SV_MAC_STEP(A, B) "v_mad_u64_u32 %0, vcc, " A ", " B ", %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
__device__ __forceinline__ void mac_carry(uint64_t& acc, uint32_t& ovf, uint32_t a, uint32_t b) {
  asm(SV_MAC_STEP("%2", "%3") : "+v"(acc), "+v"(ovf) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void mac_carry2(uint64_t& acc, uint32_t& ovf, uint32_t a0, uint32_t b0, uint32_t a1,
                                           uint32_t b1) {
  asm(SV_MAC_STEP("%2", "%3") SV_MAC_STEP("%4", "%5")
      : "+v"(acc), "+v"(ovf) : "v"(a0), "v"(b0), "v"(a1), "v"(b1) : "vcc");
}
__device__ __forceinline__ void mac_carry4(uint64_t& acc, uint32_t& ovf, const uint32_t* x, const uint32_t* y) {
  asm(SV_MAC_STEP("%2", "%3") SV_MAC_STEP("%4", "%5") SV_MAC_STEP("%6", "%7") SV_MAC_STEP("%8", "%9")
      : "+v"(acc), "+v"(ovf)
      : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3])
      : "vcc");
}
// Column-opening forms: the first product's carry initialises ovf (v_cndmask from VCC) instead of
// a v_mov of 0 before the column -- one instruction less per column (16 per multiplication).
#define SV_MAC_FIRST(A, B) "v_mad_u64_u32 %0, vcc, " A ", " B ", %0\n\tv_cndmask_b32_e64 %1, 0, 1, vcc\n\t"
__device__ __forceinline__ void mac_first(uint64_t& acc, uint32_t& ovf, uint32_t a, uint32_t b) {
  asm(SV_MAC_FIRST("%2", "%3") : "+v"(acc), "=v"(ovf) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void mac_first2(uint64_t& acc, uint32_t& ovf, uint32_t a0, uint32_t b0, uint32_t a1,
                                           uint32_t b1) {
  asm(SV_MAC_FIRST("%2", "%3") SV_MAC_STEP("%4", "%5")
      : "+v"(acc), "=&v"(ovf) : "v"(a0), "v"(b0), "v"(a1), "v"(b1) : "vcc");
}
__device__ __forceinline__ void mac_first4(uint64_t& acc, uint32_t& ovf, const uint32_t* x, const uint32_t* y) {
  asm(SV_MAC_FIRST("%2", "%3") SV_MAC_STEP("%4", "%5") SV_MAC_STEP("%6", "%7") SV_MAC_STEP("%8", "%9")
      : "+v"(acc), "=&v"(ovf)
      : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3])
      : "vcc");
}
#undef SV_MAC_FIRST
#undef SV_MAC_STEP

// Montgomery multiplication by finely integrated product scanning: column k accumulates
// a_i b_{k-i} and m_i p_{k-i} in (acc, ovf); for k < 8 the column's low word fixes m_k.
// kReduce = false skips the final conditional subtraction (fe_mul_lazy).
template <class M, bool kReduce>
SV_HD Fe<M> mont_mul(const Fe<M>& a, const Fe<M>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    // the column's products (a_i b_{k-i}, then m_i p_{k-i}); counts are compile-time constants
    uint32_t xs[16], ys[16];
    int c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (j >= 0 && j < 8) {
        xs[c] = a.v[i];
        ys[c] = b.v[j];
        c++;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 8) {
        xs[c] = m[i];
        ys[c] = M::p(j);
        c++;
      }
    }
    // the column's first asm block opens ovf (mac_first*); a column with no products before the
    // m_k step (k = 0) opens it there; the empty last column (k = 15) sets it to 0
    int q = 0;
    bool open = false;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
      open = true;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
      open = true;
    } else if (c == 1) {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
      open = true;
    }
#pragma unroll
    for (; q + 3 < c; q += 4) mac_carry4(acc, ovf, xs + q, ys + q);
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    if (k < 8) {
      m[k] = (uint32_t)acc * M::NP0;
      if (open) mac_carry(acc, ovf, m[k], M::p(0));
      else mac_first(acc, ovf, m[k], M::p(0));
    } else {
      t[k - 8] = (uint32_t)acc;
      if (!open) ovf = 0;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  const uint32_t top = (uint32_t)acc;
  if constexpr (!kReduce) {
    Fe<M> r;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = t[j];
    (void)top;
    return r;
  }
  Fe<M> d;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint64_t s = (uint64_t)t[j] - M::p(j) - br;
    d.v[j] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  const bool ge = (top != 0) || (br == 0);
  Fe<M> r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = ge ? d.v[j] : t[j];
  return r;
}
template <class M>
SV_HD Fe<M> operator*(const Fe<M>& a, const Fe<M>& b) {
  return mont_mul<M, true>(a, b);
}
// Montgomery product WITHOUT the final conditional subtraction: for a, b < 2p the result is below
// 2p (4 p^2 < 2^256 p), which is all a lazily reduced consumer needs (the decider's lane sums).
template <class M>
SV_HD Fe<M> fe_mul_lazy(const Fe<M>& a, const Fe<M>& b) {
  return mont_mul<M, false>(a, b);
}
#else
// CIOS Montgomery multiplication (host build of the same templates): r = a * b * 2^-256 mod m.
template <class M>
SV_HD Fe<M> operator*(const Fe<M>& a, const Fe<M>& b) {
  uint32_t t[10];
#pragma unroll
  for (int j = 0; j < 10; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      uint64_t s = (uint64_t)a.v[j] * b.v[i] + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    uint64_t s = (uint64_t)t[8] + c;
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    uint32_t m = t[0] * M::NP0;
    s = (uint64_t)m * M::p(0) + t[0];
    c = s >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      s = (uint64_t)m * M::p(j) + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[8] + c;
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  Fe<M> d;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint64_t s = (uint64_t)t[j] - M::p(j) - br;
    d.v[j] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  bool ge = (t[8] != 0) || (br == 0);
  Fe<M> r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = ge ? d.v[j] : t[j];
  return r;
}
template <class M>
SV_HD Fe<M> fe_mul_lazy(const Fe<M>& a, const Fe<M>& b) {
  return a * b;
}
#endif

#if defined(__HIP_DEVICE_COMPILE__)
// Montgomery squaring for throughput-bound code (many waves per SIMD: bucket accumulation, Poseidon):
// the 28 off-diagonal products a_i a_j (i < j) are scanned once into a 512-bit
// half product, doubled by one funnel shift per word, and folded into the same product-scanning
// Montgomery pass as operator* with the 8 diagonal squares (100 instead of 128 v_mad_u64_u32).
// The column carry entering the main pass stays below 2^36 (at most 9 products per column), so
// adding a doubled word cannot overflow the 64-bit accumulator.  Measured: k_accumulate 1.52 ->
// 1.49 ms at 2^20; single-wave chains (decider, batched Horner) were ~1 % slower with it (two
// dependent scans), so fe_sqr stays a * a and only the XYZZ formulas and Poseidon use fe_sqr_hp.
template <class M, bool kReduce = true>
SV_HD Fe<M> fe_sqr_hp(const Fe<M>& a) {
  uint32_t od[16];
  uint64_t acc = 0;
  uint32_t ovf = 0;
  od[0] = 0;
#pragma unroll
  for (int k = 1; k < 14; k++) {
    uint32_t xs[4], ys[4];
    int c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < j && j < 8) {
        xs[c] = a.v[i];
        ys[c] = a.v[j];
        c++;
      }
    }
    int q;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
    } else {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
    }
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    od[k] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  od[14] = (uint32_t)acc;
  od[15] = (uint32_t)(acc >> 32);
  uint32_t d[16];
  d[0] = 0;
#pragma unroll
  for (int k = 1; k < 16; k++) d[k] = __builtin_amdgcn_alignbit(od[k], od[k - 1], 31);

  uint32_t m[8], t[8];
  acc = 0;
  ovf = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    acc += d[k];
    uint32_t xs[9], ys[9];
    int c = 0;
    if ((k & 1) == 0 && k < 16) {
      xs[c] = a.v[k >> 1];
      ys[c] = a.v[k >> 1];
      c++;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 8) {
        xs[c] = m[i];
        ys[c] = M::p(j);
        c++;
      }
    }
    int q = 0;
    bool open = false;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
      open = true;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
      open = true;
    } else if (c == 1) {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
      open = true;
    }
#pragma unroll
    for (; q + 3 < c; q += 4) mac_carry4(acc, ovf, xs + q, ys + q);
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    if (k < 8) {
      m[k] = (uint32_t)acc * M::NP0;
      if (open) mac_carry(acc, ovf, m[k], M::p(0));
      else mac_first(acc, ovf, m[k], M::p(0));
    } else {
      t[k - 8] = (uint32_t)acc;
      if (!open) ovf = 0;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  const uint32_t top = (uint32_t)acc;
  if constexpr (!kReduce) {  // [0, 2p) for inputs below 2p (fe_mul_lazy)
    Fe<M> r;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = t[j];
    (void)top;
    return r;
  }
  Fe<M> dd;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint64_t s = (uint64_t)t[j] - M::p(j) - br;
    dd.v[j] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  const bool ge = (top != 0) || (br == 0);
  Fe<M> r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = ge ? dd.v[j] : t[j];
  return r;
}
#else
template <class M, bool kReduce = true>
SV_HD Fe<M> fe_sqr_hp(const Fe<M>& a) {
  return a * a;
}
#endif

// ---- the 2p domain: values in [0, 2p), as lazily reduced chains keep them (k_accumulate's
// bucket additions, the decider's lane products).  2p < 2^255 for both BN254 moduli.
template <class M>
SV_HD uint32_t p2_limb(int i) {
  return (M::p(i) << 1) | (i ? M::p(i - 1) >> 31 : 0u);
}
// carry chains through the clang builtins (v_addc / v_subb on the device); 64-bit C for g++
SV_HD uint32_t sv_addc(uint32_t a, uint32_t b, uint32_t c, uint32_t* co) {
#if defined(__clang__)
  return __builtin_addc(a, b, c, co);
#else
  const uint64_t s = (uint64_t)a + b + c;
  *co = (uint32_t)(s >> 32);
  return (uint32_t)s;
#endif
}
SV_HD uint32_t sv_subc(uint32_t a, uint32_t b, uint32_t c, uint32_t* co) {
#if defined(__clang__)
  return __builtin_subc(a, b, c, co);
#else
  const uint64_t s = (uint64_t)a - b - c;
  *co = (uint32_t)(s >> 63);
  return (uint32_t)s;
#endif
}
// a - b for a, b in [0, 2p): + 2p on borrow
template <class M>
SV_HD Fe<M> fe_sub2p(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> t, r;
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = sv_subc(a.v[i], b.v[i], br, &br);
  const uint32_t mask = 0u - br;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = sv_addc(t.v[i], p2_limb<M>(i) & mask, c, &c);
  return r;
}
// a + b for a, b in [0, 2p): - 2p when the sum reaches 2p (4p < 2^256: no carry out)
template <class M>
SV_HD Fe<M> fe_add2p(const Fe<M>& a, const Fe<M>& b) {
  Fe<M> t, d, r;
  uint32_t c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t.v[i] = sv_addc(a.v[i], b.v[i], c, &c);
    d.v[i] = sv_subc(t.v[i], p2_limb<M>(i), br, &br);
  }
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = br ? t.v[i] : d.v[i];
  return r;
}
// 2p - a for a in [0, 2p]
template <class M>
SV_HD Fe<M> fe_neg2p(const Fe<M>& a) {
  Fe<M> r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = sv_subc(p2_limb<M>(i), a.v[i], br, &br);
  return r;
}
// [0, 2p) -> [0, p)
template <class M>
SV_HD Fe<M> fe_canon2p(const Fe<M>& a) {
  Fe<M> d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d.v[i] = sv_subc(a.v[i], M::p(i), br, &br);
  return br ? a : d;
}
// a == 0 (mod p) for a in [0, 2p)
template <class M>
SV_HD bool fe_is_zero2p(const Fe<M>& a) {
  uint32_t z = 0, e = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    z |= a.v[i];
    e |= a.v[i] ^ M::p(i);
  }
  return z == 0 || e == 0;
}

template <class M>
SV_HD Fe<M> fe_sqr(const Fe<M>& a) {
  return a * a;
}

#if defined(__HIP_DEVICE_COMPILE__)
// Sum of N Montgomery products with ONE reduction: column k of the product scan accumulates
// a_n,i b_n,k-i for every pair n and then m_i p_k-i, so N products cost 64 N + 64 multiply-adds
// instead of 128 N.  With p < 2^254 the scanned value is below (N p^2 + 2^256 p) / 2^256 < 2p for
// N <= 3, so the single conditional subtraction of operator* still reduces fully.
// kReduce = false returns the scanned value itself (below 2^256 for the operand bounds the caller
// states; no final subtraction), as fe_mul_lazy does for one product.
template <class M, int N, bool kReduce = true>
SV_HD Fe<M> fe_mul_sum(const Fe<M> (&a)[N], const Fe<M> (&b)[N]) {
  static_assert(N >= 1 && N <= 3, "fe_mul_sum: the final subtraction covers N <= 3");
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t ovf = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    uint32_t xs[8 * N + 8], ys[8 * N + 8];
    int c = 0;
#pragma unroll
    for (int n = 0; n < N; n++)
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const int j = k - i;
        if (j >= 0 && j < 8) {
          xs[c] = a[n].v[i];
          ys[c] = b[n].v[j];
          c++;
        }
      }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 8) {
        xs[c] = m[i];
        ys[c] = M::p(j);
        c++;
      }
    }
    int q = 0;
    bool open = false;
    if (c >= 4) {
      mac_first4(acc, ovf, xs, ys);
      q = 4;
      open = true;
    } else if (c >= 2) {
      mac_first2(acc, ovf, xs[0], ys[0], xs[1], ys[1]);
      q = 2;
      open = true;
    } else if (c == 1) {
      mac_first(acc, ovf, xs[0], ys[0]);
      q = 1;
      open = true;
    }
#pragma unroll
    for (; q + 3 < c; q += 4) mac_carry4(acc, ovf, xs + q, ys + q);
#pragma unroll
    for (; q + 1 < c; q += 2) mac_carry2(acc, ovf, xs[q], ys[q], xs[q + 1], ys[q + 1]);
#pragma unroll
    for (; q < c; q++) mac_carry(acc, ovf, xs[q], ys[q]);
    if (k < 8) {
      m[k] = (uint32_t)acc * M::NP0;
      if (open) mac_carry(acc, ovf, m[k], M::p(0));
      else mac_first(acc, ovf, m[k], M::p(0));
    } else {
      t[k - 8] = (uint32_t)acc;
      if (!open) ovf = 0;
    }
    acc = (acc >> 32) | ((uint64_t)ovf << 32);
  }
  if constexpr (!kReduce) {
    Fe<M> r;
#pragma unroll
    for (int j = 0; j < 8; j++) r.v[j] = t[j];
    return r;
  }
  const uint32_t top = (uint32_t)acc;
  Fe<M> d;
  uint64_t br = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    uint64_t s = (uint64_t)t[j] - M::p(j) - br;
    d.v[j] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  const bool ge = (top != 0) || (br == 0);
  Fe<M> r;
#pragma unroll
  for (int j = 0; j < 8; j++) r.v[j] = ge ? d.v[j] : t[j];
  return r;
}
#else
template <class M, int N, bool kReduce = true>
SV_HD Fe<M> fe_mul_sum(const Fe<M> (&a)[N], const Fe<M> (&b)[N]) {
  Fe<M> r = a[0] * b[0];
  for (int n = 1; n < N; n++) r = r + a[n] * b[n];
  return r;
}
#endif

template <class M>
SV_HD Fe<M> fe_to_mont(const Fe<M>& a) {
  Fe<M> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = M::r2(i);
  return a * r2;
}

template <class M>
SV_HD Fe<M> fe_from_mont(const Fe<M>& a) {
  Fe<M> o = Fe<M>::zero();
  o.v[0] = 1;
  return a * o;
}

// Multi-word helpers of the binary EEA inversion fe_inv_eea (kept as the host cross-check of fe_inv).
namespace detail {
SV_HD bool lw_is_one(const uint32_t* x) {
  uint32_t acc = x[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 8; i++) acc |= x[i];
  return acc == 0;
}
SV_HD void lw_shr1(uint32_t* x, uint32_t top) {
#pragma unroll
  for (int i = 0; i < 7; i++) x[i] = (x[i] >> 1) | (x[i + 1] << 31);
  x[7] = (x[7] >> 1) | (top << 31);
}
// x = (x even ? x : x + m) / 2   (x < m < 2^255)
template <class M>
SV_HD void lw_half_mod(uint32_t* x) {
  if (x[0] & 1) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (uint64_t)x[i] + M::p(i);
      x[i] = (uint32_t)c;
      c >>= 32;
    }
    lw_shr1(x, (uint32_t)c);
  } else {
    lw_shr1(x, 0);
  }
}
SV_HD bool lw_ge(const uint32_t* a, const uint32_t* b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a[i] - b[i] - br;
    br = (s >> 63) & 1;
  }
  return br == 0;
}
SV_HD void lw_sub(uint32_t* a, const uint32_t* b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
}
// a = a - b mod m, a, b < m
template <class M>
SV_HD void lw_sub_mod(uint32_t* a, const uint32_t* b) {
  uint64_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t s = (uint64_t)a[i] - b[i] - br;
    a[i] = (uint32_t)s;
    br = (s >> 63) & 1;
  }
  if (br) {
    uint64_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      c += (uint64_t)a[i] + M::p(i);
      a[i] = (uint32_t)c;
      c >>= 32;
    }
  }
}
}  // namespace detail

// Inverse by batched divsteps (Bernstein-Yang "safegcd", variable-time form; restated from the
// published algorithm): the low 32 bits of (f, g) drive up to 30 divsteps at a time, collected in a
// 2x2 transition matrix that is then applied to the full-width (f, g) and to the Bezout
// coefficients (d, e) mod m -- ~20 matrix applications of 9 signed 30-bit limbs instead of ~500
// multi-word shift / subtract steps of the binary EEA.
// Inputs are public verifier data, so the data-dependent running time is harmless.
namespace detail {
struct S30 {
  int32_t v[9];
};
template <class M>
struct ModInv30 {
  S30 m;          // modulus in signed 30-bit limbs
  uint32_t inv;   // modulus^-1 mod 2^30
};
constexpr uint32_t kM30 = 0x3fffffffu;
template <class M>
SV_HD S30 to_s30(const uint32_t* x) {
  S30 r;
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc |= (uint64_t)x[i] << bits;
    bits += 32;
    while (bits >= 30) {
      r.v[k++] = (int32_t)(acc & kM30);
      acc >>= 30;
      bits -= 30;
    }
  }
  r.v[8] = (int32_t)acc;  // 256 - 240 = 16 bits
  return r;
}
SV_HD void from_s30(const S30& a, uint32_t* x) {  // a in [0, m), limbs normalised
  uint64_t acc = 0;
  int bits = 0, k = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc |= (uint64_t)(uint32_t)a.v[i] << bits;
    bits += 30;
    if (bits >= 32) {
      x[k++] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  if (k < 8) x[k] = (uint32_t)acc;
}
struct Trans {
  int32_t u, v, q, r;
};
// up to 30 divsteps on the low words; returns the new eta (= -delta); t * [f, g] = 2^30 [f', g']
SV_HD int32_t divsteps30(int32_t eta, uint32_t f0, uint32_t g0, Trans* t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t f = f0, g = g0;
  int i = 30;
  for (;;) {
    // divide g by 2 as often as possible (at most i more steps)
    const uint32_t gs = g | (0xffffffffu << i);
    const int zeros = __builtin_ctz(gs);
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // delta > 0: (f, g) <- (g, -f)
      eta = -eta;
      uint32_t tmp = f;
      f = g;
      g = 0u - tmp;
      tmp = u;
      u = q;
      q = 0u - tmp;
      tmp = v;
      v = r;
      r = 0u - tmp;
    }
    // cancel the bottom min(eta + 1, i, 12) bits of g with a multiple of f (f odd)
    int limit = eta + 1 > i ? i : eta + 1;
    if (limit > 12) limit = 12;
    const uint32_t m = 0xffffffffu >> (32 - limit);
    uint32_t finv = f;                 // f^-1 mod 2^3
    finv *= 2u - f * finv;             // mod 2^6
    finv *= 2u - f * finv;             // mod 2^12
    const uint32_t w = (0u - g * finv) & m;
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t->u = (int32_t)u;
  t->v = (int32_t)v;
  t->q = (int32_t)q;
  t->r = (int32_t)r;
  return eta;
}
// [f, g] <- t [f, g] / 2^30 over the first len limbs
SV_HD void update_fg(int len, S30& f, S30& g, const Trans& t) {
  int64_t cf = (int64_t)t.u * f.v[0] + (int64_t)t.v * g.v[0];
  int64_t cg = (int64_t)t.q * f.v[0] + (int64_t)t.r * g.v[0];
  cf >>= 30;
  cg >>= 30;
  for (int i = 1; i < len; i++) {
    cf += (int64_t)t.u * f.v[i] + (int64_t)t.v * g.v[i];
    cg += (int64_t)t.q * f.v[i] + (int64_t)t.r * g.v[i];
    f.v[i - 1] = (int32_t)((uint32_t)cf & kM30);
    g.v[i - 1] = (int32_t)((uint32_t)cg & kM30);
    cf >>= 30;
    cg >>= 30;
  }
  f.v[len - 1] = (int32_t)cf;
  g.v[len - 1] = (int32_t)cg;
}
// [d, e] <- (t [d, e] + m [md, me]) / 2^30 with md, me chosen to clear the low 30 bits; d, e stay
// in (-2m, m)
SV_HD void update_de(S30& d, S30& e, const Trans& t, const S30& mod, uint32_t minv) {
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se);
  int32_t me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d.v[0] + (int64_t)t.v * e.v[0];
  int64_t ce = (int64_t)t.q * d.v[0] + (int64_t)t.r * e.v[0];
  md -= (int32_t)((minv * (uint32_t)cd + (uint32_t)md) & kM30);
  me -= (int32_t)((minv * (uint32_t)ce + (uint32_t)me) & kM30);
  cd += (int64_t)mod.v[0] * md;
  ce += (int64_t)mod.v[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)t.u * d.v[i] + (int64_t)t.v * e.v[i] + (int64_t)mod.v[i] * md;
    ce += (int64_t)t.q * d.v[i] + (int64_t)t.r * e.v[i] + (int64_t)mod.v[i] * me;
    d.v[i - 1] = (int32_t)((uint32_t)cd & kM30);
    e.v[i - 1] = (int32_t)((uint32_t)ce & kM30);
    cd >>= 30;
    ce >>= 30;
  }
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}
// r in (-2m, m) -> (sign < 0 ? -r : r) mod m in [0, m), limbs normalised
SV_HD void normalize30(S30& r, int32_t sign, const S30& mod) {
  int32_t add = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += mod.v[i] & add;
  const int32_t neg = sign >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] = (r.v[i] ^ neg) - neg;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= (int32_t)kM30;
  }
  add = r.v[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r.v[i] += mod.v[i] & add;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i + 1] += r.v[i] >> 30;
    r.v[i] &= (int32_t)kM30;
  }
}
// raw integer inverse x^-1 mod m (x in [1, m))
template <class M>
SV_HD void inv_raw(const uint32_t* x, uint32_t* out) {
  uint32_t mw[8];
#pragma unroll
  for (int i = 0; i < 8; i++) mw[i] = M::p(i);
  const S30 mod = to_s30<M>(mw);
  uint32_t minv = mw[0];  // m^-1 mod 2^30 by Newton from m (odd)
#pragma unroll
  for (int k = 0; k < 5; k++) minv *= 2u - mw[0] * minv;
  minv &= kM30;
  S30 d{}, e{}, f = mod, g = to_s30<M>(x);
  e.v[0] = 1;
  int len = 9;
  int32_t eta = -1;
  for (;;) {
    Trans t;
    eta = divsteps30(eta, (uint32_t)f.v[0], (uint32_t)g.v[0], &t);
    update_de(d, e, t, mod, minv);
    update_fg(len, f, g, t);
    if (g.v[0] == 0) {
      int32_t any = 0;
      for (int j = 1; j < len; j++) any |= g.v[j];
      if (any == 0) break;
    }
    const int32_t fn = f.v[len - 1], gn = g.v[len - 1];
    int32_t cond = (len - 2) >> 31;
    cond |= fn ^ (fn >> 31);
    cond |= gn ^ (gn >> 31);
    if (cond == 0) {  // top limbs are sign-only: shorten
      f.v[len - 2] |= (int32_t)((uint32_t)fn << 30);
      g.v[len - 2] |= (int32_t)((uint32_t)gn << 30);
      len--;
    }
  }
  normalize30(d, f.v[len - 1], mod);
  from_s30(d, out);
}
}  // namespace detail

template <class M>
SV_NOINL Fe<M> fe_inv(const Fe<M>& a) {
  if (a.is_zero()) return a;
  Fe<M> r, r2;
  detail::inv_raw<M>(a.v, r.v);  // (aR)^-1
#pragma unroll
  for (int i = 0; i < 8; i++) r2.v[i] = M::r2(i);
  return r * (r2 * r2);  // (aR)^-1 * R^3 / R = a^-1 R
}

// Reference inversion (Guide to ECC alg. 2.22, binary EEA on the raw integer aR, ~2 x 254 shift /
// subtract steps): tools/hostcheck_inv.cpp checks fe_inv against it.
template <class M>
SV_NOINL Fe<M> fe_inv_eea(const Fe<M>& a) {
  if (a.is_zero()) return a;
  uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    u[i] = a.v[i];
    v[i] = M::p(i);
    x1[i] = i == 0 ? 1u : 0u;
    x2[i] = 0u;
  }
  // invariants: x1 * a == u, x2 * a == v (mod m); gcd(u, v) == 1
  while (!detail::lw_is_one(u) && !detail::lw_is_one(v)) {
    while (!(u[0] & 1)) {
      detail::lw_shr1(u, 0);
      detail::lw_half_mod<M>(x1);
    }
    while (!(v[0] & 1)) {
      detail::lw_shr1(v, 0);
      detail::lw_half_mod<M>(x2);
    }
    if (detail::lw_ge(u, v)) {
      detail::lw_sub(u, v);
      detail::lw_sub_mod<M>(x1, x2);
    } else {
      detail::lw_sub(v, u);
      detail::lw_sub_mod<M>(x2, x1);
    }
  }
  Fe<M> r, r2;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.v[i] = detail::lw_is_one(u) ? x1[i] : x2[i];
    r2.v[i] = M::r2(i);
  }
  return r * (r2 * r2);  // (aR)^-1 * R^3 / R = a^-1 R
}

using Fq = Fe<FqTag>;
using Fr = Fe<FrTag>;

SV_HD Fq fq_const(const uint32_t (&c)[8]) {
  Fq r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = c[i];
  return r;
}

// ------------------------------------------------------------------------------------------
// Fq2 = Fq[u]/(u^2+1)
// ------------------------------------------------------------------------------------------
struct Fq2 {
  Fq c0, c1;
  SV_HD static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  SV_HD static Fq2 one() { return {Fq::one(), Fq::zero()}; }
  SV_HD bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  SV_HD bool operator==(const Fq2& o) const { return c0 == o.c0 && c1 == o.c1; }
};

#if defined(__HIP_DEVICE_COMPILE__)
// both components' chains in one loop (four independent carry chains interleave, see Fe add)
SV_HD Fq2 operator+(const Fq2& a, const Fq2& b) {
  Fq t0, t1, d0, d1;
  uint32_t c0 = 0, c1 = 0, e0 = 0, e1 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t0.v[i] = __builtin_addc(a.c0.v[i], b.c0.v[i], c0, &c0);
    t1.v[i] = __builtin_addc(a.c1.v[i], b.c1.v[i], c1, &c1);
    d0.v[i] = __builtin_subc(t0.v[i], FQ_P[i], e0, &e0);
    d1.v[i] = __builtin_subc(t1.v[i], FQ_P[i], e1, &e1);
  }
  Fq2 r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.c0.v[i] = e0 ? t0.v[i] : d0.v[i];
    r.c1.v[i] = e1 ? t1.v[i] : d1.v[i];
  }
  return r;
}
SV_HD Fq2 operator-(const Fq2& a, const Fq2& b) {
  Fq t0, t1, w0, w1, u0, u1;
  uint32_t b0 = 0, b1 = 0, x0 = 0, x1 = 0, c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t0.v[i] = __builtin_subc(a.c0.v[i], b.c0.v[i], b0, &b0);
    t1.v[i] = __builtin_subc(a.c1.v[i], b.c1.v[i], b1, &b1);
    w0.v[i] = __builtin_subc(FQ_P[i], b.c0.v[i], x0, &x0);
    w1.v[i] = __builtin_subc(FQ_P[i], b.c1.v[i], x1, &x1);
    u0.v[i] = __builtin_addc(a.c0.v[i], w0.v[i], c0, &c0);
    u1.v[i] = __builtin_addc(a.c1.v[i], w1.v[i], c1, &c1);
  }
  Fq2 r;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.c0.v[i] = b0 ? u0.v[i] : t0.v[i];
    r.c1.v[i] = b1 ? u1.v[i] : t1.v[i];
  }
  return r;
}
#else
SV_HD Fq2 operator+(const Fq2& a, const Fq2& b) { return {a.c0 + b.c0, a.c1 + b.c1}; }
SV_HD Fq2 operator-(const Fq2& a, const Fq2& b) { return {a.c0 - b.c0, a.c1 - b.c1}; }
#endif
SV_HD Fq2 operator-(const Fq2& a) { return {-a.c0, -a.c1}; }
SV_HD Fq2 operator*(const Fq2& a, const Fq2& b) {
  Fq t0 = a.c0 * b.c0;
  Fq t1 = a.c1 * b.c1;
  Fq t2 = (a.c0 + a.c1) * (b.c0 + b.c1);
  return {t0 - t1, t2 - t0 - t1};
}
SV_HD Fq2 operator*(const Fq2& a, const Fq& s) { return {a.c0 * s, a.c1 * s}; }
SV_HD Fq2 fq2_sqr(const Fq2& a) {
  // (a0 + a1)(a0 - a1), 2 a0 a1
  Fq t = a.c0 * a.c1;
  return {(a.c0 + a.c1) * (a.c0 - a.c1), t + t};
}
SV_HD Fq2 fq2_dbl(const Fq2& a) { return a + a; }
SV_HD Fq2 fq2_conj(const Fq2& a) { return {a.c0, -a.c1}; }
SV_HD Fq2 fq2_mul_xi(const Fq2& a) {
  // (a0 + a1 u)(9 + u) = (9 a0 - a1) + (a0 + 9 a1) u
  Fq a0_2 = a.c0 + a.c0, a1_2 = a.c1 + a.c1;
  Fq a0_4 = a0_2 + a0_2, a1_4 = a1_2 + a1_2;
  Fq a0_8 = a0_4 + a0_4, a1_8 = a1_4 + a1_4;
  return {a0_8 + a.c0 - a.c1, a1_8 + a.c1 + a.c0};
}
SV_NOINL Fq2 fq2_inv(const Fq2& a) {
  Fq t = fe_inv(fe_sqr(a.c0) + fe_sqr(a.c1));
  return {a.c0 * t, -(a.c1 * t)};
}
SV_HD Fq2 fq2_const(const uint32_t (&c0)[8], const uint32_t (&c1)[8]) {
  return {fq_const(c0), fq_const(c1)};
}

// ------------------------------------------------------------------------------------------
// Fq6 = Fq2[v]/(v^3 - xi),  Fq12 = Fq6[w]/(w^2 - v)
// ------------------------------------------------------------------------------------------
struct Fq6 {
  Fq2 c0, c1, c2;
  SV_HD static Fq6 zero() { return {Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
  SV_HD static Fq6 one() { return {Fq2::one(), Fq2::zero(), Fq2::zero()}; }
  SV_HD bool operator==(const Fq6& o) const { return c0 == o.c0 && c1 == o.c1 && c2 == o.c2; }
};

SV_HD Fq6 operator+(const Fq6& a, const Fq6& b) { return {a.c0 + b.c0, a.c1 + b.c1, a.c2 + b.c2}; }
SV_HD Fq6 operator-(const Fq6& a, const Fq6& b) { return {a.c0 - b.c0, a.c1 - b.c1, a.c2 - b.c2}; }
SV_HD Fq6 operator-(const Fq6& a) { return {-a.c0, -a.c1, -a.c2}; }
SV_NOINL Fq6 operator*(const Fq6& a, const Fq6& b) {
  Fq2 t0 = a.c0 * b.c0, t1 = a.c1 * b.c1, t2 = a.c2 * b.c2;
  Fq2 c0 = t0 + fq2_mul_xi((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2);
  Fq2 c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + fq2_mul_xi(t2);
  Fq2 c2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1;
  return {c0, c1, c2};
}
SV_HD Fq6 fq6_mul_by_v(const Fq6& a) { return {fq2_mul_xi(a.c2), a.c0, a.c1}; }
SV_NOINL Fq6 fq6_sqr(const Fq6& a) {
  // CH-SQR2
  Fq2 s0 = fq2_sqr(a.c0);
  Fq2 ab = a.c0 * a.c1;
  Fq2 s1 = fq2_dbl(ab);
  Fq2 s2 = fq2_sqr(a.c0 - a.c1 + a.c2);
  Fq2 bc = a.c1 * a.c2;
  Fq2 s3 = fq2_dbl(bc);
  Fq2 s4 = fq2_sqr(a.c2);
  return {s0 + fq2_mul_xi(s3), s1 + fq2_mul_xi(s4), s1 + s2 + s3 - s0 - s4};
}
// a * (b0 + b1 v)
SV_NOINL Fq6 fq6_mul_by_01(const Fq6& a, const Fq2& b0, const Fq2& b1) {
  Fq2 aa = a.c0 * b0, bb = a.c1 * b1;
  Fq2 t1 = fq2_mul_xi(a.c2 * b1) + aa;
  Fq2 t2 = (b0 + b1) * (a.c0 + a.c1) - aa - bb;
  Fq2 t3 = a.c2 * b0 + bb;
  return {t1, t2, t3};
}
SV_NOINL Fq6 fq6_mul_fq2(const Fq6& a, const Fq2& s) { return {a.c0 * s, a.c1 * s, a.c2 * s}; }
SV_NOINL Fq6 fq6_inv(const Fq6& a) {
  Fq2 t0 = fq2_sqr(a.c0) - fq2_mul_xi(a.c1 * a.c2);
  Fq2 t1 = fq2_mul_xi(fq2_sqr(a.c2)) - a.c0 * a.c1;
  Fq2 t2 = fq2_sqr(a.c1) - a.c0 * a.c2;
  Fq2 d = a.c0 * t0 + fq2_mul_xi(a.c2 * t1 + a.c1 * t2);
  Fq2 di = fq2_inv(d);
  return {t0 * di, t1 * di, t2 * di};
}

struct Fq12 {
  Fq6 c0, c1;
  SV_HD static Fq12 one() { return {Fq6::one(), Fq6::zero()}; }
  SV_HD bool operator==(const Fq12& o) const { return c0 == o.c0 && c1 == o.c1; }
  SV_HD bool is_one() const { return *this == one(); }
};

SV_NOINL Fq12 operator*(const Fq12& a, const Fq12& b) {
  Fq6 t0 = a.c0 * b.c0, t1 = a.c1 * b.c1;
  return {t0 + fq6_mul_by_v(t1), (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1};
}
SV_NOINL Fq12 fq12_sqr(const Fq12& a) {
  // complex squaring: c0 = (a0 + a1)(a0 + v a1) - t - v t, c1 = 2t, t = a0 a1
  Fq6 t = a.c0 * a.c1;
  Fq6 c0 = (a.c0 + a.c1) * (a.c0 + fq6_mul_by_v(a.c1)) - t - fq6_mul_by_v(t);
  return {c0, t + t};
}
SV_HD Fq12 fq12_conj(const Fq12& a) { return {a.c0, -a.c1}; }
SV_NOINL Fq12 fq12_inv(const Fq12& a) {
  Fq6 t = a.c0 * a.c0 - fq6_mul_by_v(a.c1 * a.c1);
  Fq6 ti = fq6_inv(t);
  return {a.c0 * ti, -(a.c1 * ti)};
}
// f * (c0 + c3 w + c4 v w): the sparse D-type line (positions 0, 3, 4)
SV_NOINL Fq12 fq12_mul_by_034(const Fq12& f, const Fq2& c0, const Fq2& c3, const Fq2& c4) {
  Fq6 t0 = fq6_mul_fq2(f.c0, c0);
  Fq6 t1 = fq6_mul_by_01(f.c1, c3, c4);
  Fq6 t2 = fq6_mul_by_01(f.c0 + f.c1, c0 + c3, c4) - t0 - t1;
  return {fq6_mul_by_v(t1) + t0, t2};
}

// Frobenius^n: coefficient of w^k gets conj^n(g) * GAMMAn_k.
template <int N>
SV_NOINL Fq12 fq12_frob(const Fq12& a);

#define SV_G(n, k) fq2_const(GAMMA##n##_##k##_C0, GAMMA##n##_##k##_C1)
template <>
SV_NOINL Fq12 fq12_frob<1>(const Fq12& a) {
  return {{fq2_conj(a.c0.c0), fq2_conj(a.c0.c1) * SV_G(1, 2), fq2_conj(a.c0.c2) * SV_G(1, 4)},
          {fq2_conj(a.c1.c0) * SV_G(1, 1), fq2_conj(a.c1.c1) * SV_G(1, 3), fq2_conj(a.c1.c2) * SV_G(1, 5)}};
}
template <>
SV_NOINL Fq12 fq12_frob<2>(const Fq12& a) {
  // GAMMA2_k lie in Fq (c1 = 0)
  return {{a.c0.c0, a.c0.c1 * SV_G(2, 2).c0, a.c0.c2 * SV_G(2, 4).c0},
          {a.c1.c0 * SV_G(2, 1).c0, a.c1.c1 * SV_G(2, 3).c0, a.c1.c2 * SV_G(2, 5).c0}};
}
template <>
SV_NOINL Fq12 fq12_frob<3>(const Fq12& a) {
  return {{fq2_conj(a.c0.c0), fq2_conj(a.c0.c1) * SV_G(3, 2), fq2_conj(a.c0.c2) * SV_G(3, 4)},
          {fq2_conj(a.c1.c0) * SV_G(3, 1), fq2_conj(a.c1.c1) * SV_G(3, 3), fq2_conj(a.c1.c2) * SV_G(3, 5)}};
}
#undef SV_G

}  // namespace sv
