// f2: the x^5 Poseidon sponge over BN254 Fr that drives PoseidonTranscript's Fiat-Shamir challenges
// (snark-verifier/src/util/hash/poseidon.rs, system/halo2/transcript/halo2.rs:198-227).
//
// One lane per state.  The permutation runs the reference's optimised HADES schedule
// (OptimizedPoseidonSpec, poseidon.rs:230-313; Poseidon::permutation, :469-500): the round constants
// folded through the inverse MDS (S-box then "+ constant"), a pre-sparse MDS after the first full
// half, and in each of the R_P partial rounds a sparse matrix (row . state -> state[0], state[i] +=
// col_hat[i-1] * state[0]) instead of the dense MDS: 2 t - 1 products per partial round instead of
// t^2.  The constants come from oracle/poseidon.py's restatement of the Grain-LFSR generator and of
// the reference's factorisation (tools/gen_consts.py -> poseidon_consts.hpp, Montgomery limbs); the
// schedule computes the same map as the plain ARC -> S-box -> MDS rounds (pinned by the reference's
// permutation KATs, tests.rs:34-85).  All constant loads are wave-uniform (scalar loads); each
// lane's state stays in VGPRs.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "field.hpp"
#include "field29.hpp"
#include "poseidon.hpp"
#include "poseidon_consts.hpp"
#include "runtime.hpp"

namespace sv {

__constant__ uint32_t c_start3[] = SV_POSEIDON_T3_START_INIT;
__constant__ uint32_t c_partial3[] = SV_POSEIDON_T3_PARTIAL_INIT;
__constant__ uint32_t c_end3[] = SV_POSEIDON_T3_END_INIT;
__constant__ uint32_t c_mds3[] = SV_POSEIDON_T3_MDS_INIT;
__constant__ uint32_t c_pre3[] = SV_POSEIDON_T3_PRE_INIT;
__constant__ uint32_t c_sparse3[] = SV_POSEIDON_T3_SPARSE_INIT;
__constant__ uint32_t c_start3_29[] = SV_POSEIDON_T3_START_R29_INIT;
__constant__ uint32_t c_partial3_29[] = SV_POSEIDON_T3_PARTIAL_R29_INIT;
__constant__ uint32_t c_end3_29[] = SV_POSEIDON_T3_END_R29_INIT;
__constant__ uint32_t c_mds3_29[] = SV_POSEIDON_T3_MDS_R29_INIT;
__constant__ uint32_t c_pre3_29[] = SV_POSEIDON_T3_PRE_R29_INIT;
__constant__ uint32_t c_sparse3_29[] = SV_POSEIDON_T3_SPARSE_R29_INIT;
__constant__ uint32_t c_start5[] = SV_POSEIDON_T5_START_INIT;
__constant__ uint32_t c_partial5[] = SV_POSEIDON_T5_PARTIAL_INIT;
__constant__ uint32_t c_end5[] = SV_POSEIDON_T5_END_INIT;
__constant__ uint32_t c_mds5[] = SV_POSEIDON_T5_MDS_INIT;
__constant__ uint32_t c_pre5[] = SV_POSEIDON_T5_PRE_INIT;
__constant__ uint32_t c_sparse5[] = SV_POSEIDON_T5_SPARSE_INIT;

template <int T>
struct PSpec;
template <>
struct PSpec<3> {
  static constexpr int RF = SV_POSEIDON_T3_RF, RP = SV_POSEIDON_T3_RP;
  static __device__ __forceinline__ const uint32_t* start() { return c_start3; }
  static __device__ __forceinline__ const uint32_t* partial() { return c_partial3; }
  static __device__ __forceinline__ const uint32_t* end() { return c_end3; }
  static __device__ __forceinline__ const uint32_t* mds() { return c_mds3; }
  static __device__ __forceinline__ const uint32_t* pre() { return c_pre3; }
  static __device__ __forceinline__ const uint32_t* sparse() { return c_sparse3; }
};
template <>
struct PSpec<5> {
  static constexpr int RF = SV_POSEIDON_T5_RF, RP = SV_POSEIDON_T5_RP;
  static __device__ __forceinline__ const uint32_t* start() { return c_start5; }
  static __device__ __forceinline__ const uint32_t* partial() { return c_partial5; }
  static __device__ __forceinline__ const uint32_t* end() { return c_end5; }
  static __device__ __forceinline__ const uint32_t* mds() { return c_mds5; }
  static __device__ __forceinline__ const uint32_t* pre() { return c_pre5; }
  static __device__ __forceinline__ const uint32_t* sparse() { return c_sparse5; }
};

__device__ __forceinline__ Fr ld_const(const uint32_t* p) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = p[i];
  return r;
}

// The permutation runs in field.hpp's lazily reduced domain: every state word stays below 2.32 r
// (r < 2^254 is the Fr modulus, r / R < 0.18905 for R = 2^256), so no product pays its final
// conditional subtraction.  Bounds: a Montgomery product of x, y is below x y / R + r, so
//   * pow5 of a word below 2.32 r: x^2 < 2.02 r, x^4 < 1.78 r, x^5 < 1.78 r;
//   * a t = 3 MDS row, a fused sum of three products of words below 2.32 r with constants below r,
//     scans below (3 * 2.32 * 0.18905 + 1) r < 2.316 r and is kept as scanned (no subtraction);
//   * "+ constant" after the S-box wraps at 2r (fe_add2p): 1.78 r + r - 2r < r, else below 2r;
//   * a partial round's state[i] += col_hat[i-1] * state[0] adds a product below 1.38 r and wraps
//     at 2r, so it never grows past max(2r, its previous bound).
// The last full round reduces its rows once (below 1.32 r) and the result is canonicalised.  t = 5
// rows (two fused sums and an addition) keep fe_mul_sum's subtraction.
__device__ __forceinline__ Fr pow5(const Fr& x) {
  const Fr x2 = fe_sqr_hp<FrTag, false>(x);
  return fe_mul_lazy(fe_sqr_hp<FrTag, false>(x2), x);
}

// One MDS row, sum_j s_j M_ij, as fused sums of up to three products with one Montgomery reduction
// each (fe_mul_sum): t = 3 is one reduction per row instead of three.
template <int T, bool kLazy = (T == 3)>
__device__ __forceinline__ Fr mds_row(const Fr (&s)[T], const uint32_t* row) {
  constexpr int A = T < 3 ? T : 3;
  Fr x[A], y[A];
#pragma unroll
  for (int j = 0; j < A; j++) x[j] = s[j], y[j] = ld_const(row + j * 8);
  Fr acc = fe_mul_sum<FrTag, A, !kLazy>(x, y);
  if constexpr (T > 3) {
    constexpr int B = T - 3;
    static_assert(B <= 3, "mds_row: t <= 6");
    Fr u[B], v[B];
#pragma unroll
    for (int j = 0; j < B; j++) u[j] = s[3 + j], v[j] = ld_const(row + (3 + j) * 8);
    acc = acc + fe_mul_sum(u, v);
  }
  return acc;
}

// s <- M s for a dense t x t matrix (rows of fused sums of products)
template <int T, bool kLazy = (T == 3)>
__device__ __forceinline__ void apply_mds(Fr (&s)[T], const uint32_t* m) {
  Fr o[T];
#pragma unroll
  for (int i = 0; i < T; i++) o[i] = mds_row<T, kLazy>(s, m + i * T * 8);
#pragma unroll
  for (int i = 0; i < T; i++) s[i] = o[i];
}

// full round: s_i <- s_i^5 + c_i (State::sbox_full, poseidon.rs:353-357), then the dense matrix
template <int T, bool kLazy = (T == 3)>
__device__ __forceinline__ void full_round(Fr (&s)[T], const uint32_t* c, const uint32_t* m) {
#pragma unroll
  for (int i = 0; i < T; i++) s[i] = c ? fe_add2p(pow5(s[i]), ld_const(c + i * 8)) : pow5(s[i]);
  apply_mds<T, kLazy>(s, m);
}

// Poseidon::permutation (poseidon.rs:469-500) without the absorbed inputs: the bare HADES map.
template <int T>
__device__ __forceinline__ void permute(Fr (&s)[T]) {
  constexpr int RF = PSpec<T>::RF, RP = PSpec<T>::RP, H = RF / 2;
  const uint32_t* start = PSpec<T>::start();
#pragma unroll
  for (int i = 0; i < T; i++) s[i] = s[i] + ld_const(start + i * 8);  // absorb_with_pre_constants
  for (int r = 1; r < H; r++) full_round<T>(s, start + r * T * 8, PSpec<T>::mds());
  full_round<T>(s, start + H * T * 8, PSpec<T>::pre());
  // partial rounds: sbox_part, then apply_sparse_mds (poseidon.rs:359-361, :399-412)
  const uint32_t* partial = PSpec<T>::partial();
  const uint32_t* sparse = PSpec<T>::sparse();
  for (int r = 0; r < RP; r++) {
    s[0] = fe_add2p(pow5(s[0]), ld_const(partial + r * 8));
    const uint32_t* row = sparse + r * (2 * T - 1) * 8;
    const Fr s0 = mds_row<T>(s, row);
#pragma unroll
    for (int i = 1; i < T; i++) s[i] = fe_add2p(s[i], fe_mul_lazy(s[0], ld_const(row + (T + i - 1) * 8)));
    s[0] = s0;
  }
  const uint32_t* end = PSpec<T>::end();
  for (int r = 0; r < H - 1; r++) full_round<T>(s, end + r * T * 8, PSpec<T>::mds());
  full_round<T, false>(s, nullptr, PSpec<T>::mds());  // rows reduced once: below 1.32 r
#pragma unroll
  for (int i = 0; i < T; i++) s[i] = fe_canon2p(s[i]);
}

// ---- t = 3 over field29.hpp's 9 x 29-bit limbs (round 4, default; SVGPU_POSEIDON_R29=0 keeps the
// 8 x 32-bit rounds above).  Every partial product is one v_mad_u64_u32 with no carry add, and an
// MDS row is ONE Montgomery reduction of three products (mul_sum3).  Same schedule, constants in
// the limb form (c 2^261 mod r, tools/gen_consts.py); the state enters and leaves in field.hpp's
// form.  Bounds (field29.hpp's contract, r the modulus):
//   * pow5 of a word below 12 r is below 2 r; "+ constant" makes it below 3 r (no reduction);
//   * an MDS row of words below 9 r with constants below r is below 2 r;
//   * a partial round's state[i] += col_hat[i-1] * state[0] adds a product below 2 r to a word
//     below 4 r and is brought back below 4 r (csub<4>: below 8 r in);
//   * the last full round leaves words below 2 r, made canonical on the way out (to_r32).
namespace p29 {
using E = r29::F29<r29::FrM29>;
__device__ __forceinline__ E ld(const uint32_t* p) {  // a constant (wave-uniform: scalar loads)
  E r;
#pragma unroll
  for (int i = 0; i < r29::L; i++) r.v[i] = p[i];
  return r;
}
__device__ __forceinline__ E pow5(const E& x) { return r29::mul(r29::sqr(r29::sqr(x)), x); }
// the state as three named words (an E[3] array ended up in scratch memory)
__device__ __forceinline__ E row(const E& a, const E& b, const E& c, const uint32_t* m) {
  return r29::mul_sum3(a, ld(m), b, ld(m + 9), c, ld(m + 18));
}
__device__ __forceinline__ void mds(E& a, E& b, E& c, const uint32_t* m) {
  const E o0 = row(a, b, c, m), o1 = row(a, b, c, m + 27), o2 = row(a, b, c, m + 54);
  a = o0, b = o1, c = o2;
}
__device__ __forceinline__ void full(E& a, E& b, E& c, const uint32_t* k, const uint32_t* m) {
  if (k) {
    a = r29::add(pow5(a), ld(k));
    b = r29::add(pow5(b), ld(k + 9));
    c = r29::add(pow5(c), ld(k + 18));
  } else {
    a = pow5(a), b = pow5(b), c = pow5(c);
  }
  mds(a, b, c, m);
}
__device__ __forceinline__ void permute(E& a, E& b, E& c) {
  constexpr int RF = SV_POSEIDON_T3_RF, RP = SV_POSEIDON_T3_RP, H = RF / 2;
  a = r29::add(a, ld(c_start3_29));
  b = r29::add(b, ld(c_start3_29 + 9));
  c = r29::add(c, ld(c_start3_29 + 18));
  for (int r = 1; r < H; r++) full(a, b, c, c_start3_29 + r * 27, c_mds3_29);
  full(a, b, c, c_start3_29 + H * 27, c_pre3_29);
  for (int r = 0; r < RP; r++) {
    a = r29::add(pow5(a), ld(c_partial3_29 + r * 9));
    const uint32_t* rw = c_sparse3_29 + r * 5 * 9;
    const E a2 = row(a, b, c, rw);
    b = r29::csub<4>(r29::add(b, r29::mul(a, ld(rw + 27))));
    c = r29::csub<4>(r29::add(c, r29::mul(a, ld(rw + 36))));
    a = a2;
  }
  for (int r = 0; r < H - 1; r++) full(a, b, c, c_end3_29 + r * 27, c_mds3_29);
  full(a, b, c, nullptr, c_mds3_29);
}
}  // namespace p29

// the permutation on field.hpp words (Montgomery, reduced): the 29-bit rounds for t = 3 when R29
template <int T, bool R29>
__device__ __forceinline__ void permute_sel(Fr (&s)[T]) {
  if constexpr (R29 && T == 3) {
    p29::E a = r29::to_r29<r29::FrM29>(s[0].v), b = r29::to_r29<r29::FrM29>(s[1].v),
           c = r29::to_r29<r29::FrM29>(s[2].v);
    p29::permute(a, b, c);
    r29::to_r32(a, s[0].v);
    r29::to_r32(b, s[1].v);
    r29::to_r32(c, s[2].v);
  } else {
    permute<T>(s);
  }
}

__device__ __forceinline__ Fr load_fr(const Fr* p, int mont) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1];
  Fr r;
  r.v[0] = a.x, r.v[1] = a.y, r.v[2] = a.z, r.v[3] = a.w;
  r.v[4] = b.x, r.v[5] = b.y, r.v[6] = b.z, r.v[7] = b.w;
  return mont ? r : fe_to_mont(r);
}

__device__ __forceinline__ void store_fr(Fr* p, Fr v, int mont) {
  if (!mont) v = fe_from_mont(v);
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.v[0], v.v[1], v.v[2], v.v[3]);
  q[1] = make_uint4(v.v[4], v.v[5], v.v[6], v.v[7]);
}

template <int T, bool R29>
__global__ void __launch_bounds__(256) k_poseidon_permute(Fr* __restrict__ st, uint32_t n, int mont) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr s[T];
#pragma unroll
  for (int k = 0; k < T; k++) s[k] = load_fr(st + (size_t)i * T + k, mont);
  permute_sel<T, R29>(s);
#pragma unroll
  for (int k = 0; k < T; k++) store_fr(st + (size_t)i * T + k, s[k], mont);
}

// Poseidon::squeeze (poseidon.rs:455-467) for n independent sponges: sponge j's state (t elements,
// in/out; Poseidon::new starts it at (2^64, 0, ..), poseidon.rs:335-342) absorbs its buffered
// elements el[off[j] .. off[j+1]) RATE at a time: each chunk is added into state[1..], a chunk
// shorter than RATE is padded with a single 1 (absorb_with_pre_constants, poseidon.rs:363-385),
// and the state is permuted; when the buffer length is a multiple of RATE (including 0) one more
// permutation runs on the padded empty chunk.  The challenge is state[1].  Elements must be reduced
// field elements (halo2curves' Fr always is; the Python mirror reduces its ints mod r).
template <int T, bool R29>
__global__ void __launch_bounds__(256) k_poseidon_squeeze(Fr* __restrict__ st, const Fr* __restrict__ el,
                                                         const uint64_t* __restrict__ off, uint32_t n, int mont,
                                                         Fr* __restrict__ out) {
  constexpr int RATE = T - 1;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint64_t b = off[j], e = off[j + 1];
  Fr s[T];
#pragma unroll
  for (int k = 0; k < T; k++) s[k] = load_fr(st + (size_t)j * T + k, mont);
  uint64_t p = b;
  while (p < e) {
    const uint64_t m = e - p < (uint64_t)RATE ? e - p : (uint64_t)RATE;
#pragma unroll
    for (int k = 0; k < RATE; k++) {
      if ((uint64_t)k < m) s[k + 1] = s[k + 1] + load_fr(el + p + k, mont);
      if ((uint64_t)k == m) s[k + 1] = s[k + 1] + Fr::one();  // 10* padding of a short chunk
    }
    permute_sel<T, R29>(s);
    p += m;
  }
  if ((e - b) % RATE == 0) {  // exact: one more permutation of the padded empty chunk
    s[1] = s[1] + Fr::one();
    permute_sel<T, R29>(s);
  }
#pragma unroll
  for (int k = 0; k < T; k++) store_fr(st + (size_t)j * T + k, s[k], mont);
  if (out) store_fr(out + j, s[1], mont);
}

// t = 3 on the 29-bit limbs unless SVGPU_POSEIDON_R29=0 (read per call)
static bool poseidon_r29() {
  const char* e = getenv("SVGPU_POSEIDON_R29");
  return !e || atoi(e) != 0;
}

int poseidon_permute_device(void* d_states, size_t n, int t, int form, hipStream_t st) {
  if (n == 0) return SV_OK;
  if (n > 0xffffffffull) {
    set_error("poseidon: n = %zu exceeds 2^32 - 1", n);
    return SV_ERR_LEN;
  }
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  Fr* s = static_cast<Fr*>(d_states);
  if (t == 3 && poseidon_r29())
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_permute<3, true>), dim3(blocks), dim3(256), 0, st, s, (uint32_t)n,
                       form);
  else if (t == 3)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_permute<3, false>), dim3(blocks), dim3(256), 0, st, s, (uint32_t)n,
                       form);
  else if (t == 5)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_permute<5, false>), dim3(blocks), dim3(256), 0, st, s, (uint32_t)n,
                       form);
  else {
    set_error("poseidon: unsupported width t = %d (3 or 5)", t);
    return SV_ERR_ARG;
  }
  SV_HIP(hipGetLastError());
  return SV_OK;
}

int poseidon_squeeze_device(void* d_states, const void* d_elements, const uint64_t* d_offsets, size_t n, int t,
                           int form, void* d_out, hipStream_t st) {
  if (n == 0) return SV_OK;
  if (n > 0xffffffffull) {
    set_error("poseidon: n = %zu exceeds 2^32 - 1", n);
    return SV_ERR_LEN;
  }
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  Fr* s = static_cast<Fr*>(d_states);
  const Fr* e = static_cast<const Fr*>(d_elements);
  Fr* o = static_cast<Fr*>(d_out);
  if (t == 3 && poseidon_r29())
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_squeeze<3, true>), dim3(blocks), dim3(256), 0, st, s, e, d_offsets,
                       (uint32_t)n, form, o);
  else if (t == 3)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_squeeze<3, false>), dim3(blocks), dim3(256), 0, st, s, e, d_offsets,
                       (uint32_t)n, form, o);
  else if (t == 5)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(k_poseidon_squeeze<5, false>), dim3(blocks), dim3(256), 0, st, s, e, d_offsets,
                       (uint32_t)n, form, o);
  else {
    set_error("poseidon: unsupported width t = %d (3 or 5)", t);
    return SV_ERR_ARG;
  }
  SV_HIP(hipGetLastError());
  return SV_OK;
}

}  // namespace sv
