// Device-side helpers around the hot path:
//  * deterministic synthetic inputs (SURVEY.md section 8d generator, index-addressable SplitMix64
//    streams; byte-identical to oracle/bn254.py gen_scalar / gen_base),
//  * powers of the accumulation challenge r (LoadedScalar::powers, snark-verifier/src/loader.rs:71-78)
//    for KzgAs::create_proof's two MSMs (snark-verifier/src/pcs/kzg/accumulation.rs:177-192).
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "gen.hpp"
#include "runtime.hpp"

namespace sv {

struct SplitMix {
  uint64_t s;
  __device__ uint64_t next() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
};

__device__ __forceinline__ SplitMix stream_for(uint64_t seed, uint64_t i) {
  return SplitMix{seed * 0x9E3779B97F4A7C15ull + i * 0xD1B54A32D192ED03ull};
}

template <class M>
__device__ __forceinline__ Fe<M> draw254(SplitMix& sm) {
  Fe<M> r;
  for (int k = 0; k < 4; k++) {
    uint64_t v = sm.next();
    if (k == 3) v &= (1ull << 62) - 1;
    r.v[2 * k] = (uint32_t)v;
    r.v[2 * k + 1] = (uint32_t)(v >> 32);
  }
  return r;
}

__device__ __forceinline__ void store_fe(void* dst, const uint32_t* v) {
  uint4* p = reinterpret_cast<uint4*>(dst);
  p[0] = make_uint4(v[0], v[1], v[2], v[3]);
  p[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

__global__ void k_gen_scalars(Fr* __restrict__ out, uint32_t n, uint64_t seed, uint64_t start, int mont) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  SplitMix sm = stream_for(seed, start + i);
  Fr v;
  do {
    v = draw254<FrTag>(sm);
  } while (!v.is_reduced());
  if (mont) v = fe_to_mont(v);
  store_fe(out + i, v.v);
}

__global__ void k_gen_bases(G1Aff* __restrict__ out, uint32_t n, uint64_t seed, uint64_t start, int mont) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  SplitMix sm = stream_for(seed, start + i);
  const Fq b3 = fq_const(FQ_B3);
  while (true) {
    Fq x = draw254<FqTag>(sm);
    if (!x.is_reduced()) continue;
    Fq xm = fe_to_mont(x);
    Fq rhs = fe_sqr(xm) * xm + b3;
    // y = rhs^((p+1)/4)
    Fq y = Fq::one();
    for (int li = 7; li >= 0; li--)
      for (int b = 31; b >= 0; b--) {
        y = fe_sqr_hp(y);
        if ((FQ_SQRT_EXP[li] >> b) & 1) y = y * rhs;
      }
    if (fe_sqr(y) != rhs) continue;
    uint64_t par = sm.next() & 1;
    Fq yc = fe_from_mont(y);
    if ((yc.v[0] & 1) != par) y = -y;
    G1Aff r;
    r.x = mont ? xm : x;
    r.y = mont ? y : fe_from_mont(y);
    store_fe(reinterpret_cast<char*>(out + i), r.x.v);
    store_fe(reinterpret_cast<char*>(out + i) + 32, r.y.v);
    return;
  }
}

// out[i] = r^i; `mont_in` / `mont_out` select the forms of r and of the output
__global__ void k_powers(const Fr* __restrict__ r_in, int mont_in, uint32_t n, int mont_out,
                         Fr* __restrict__ out) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr r = *r_in;
  if (!mont_in) r = fe_to_mont(r);
  Fr acc = Fr::one();
  for (int b = 31; b >= 0; b--) {
    acc = fe_sqr(acc);
    if ((i >> b) & 1) acc = acc * r;
  }
  if (!mont_out) acc = fe_from_mont(acc);
  store_fe(out + i, acc.v);
}

int gen_scalars_device(void* d, size_t n, uint64_t seed, uint64_t start, int form, int device,
                       hipStream_t user_stream) {
  if (n == 0) return SV_OK;
  WsLease lease(device, user_stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  hipStream_t st = lease.get()->stream;
  hipLaunchKernelGGL(k_gen_scalars, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<Fr*>(d), (uint32_t)n, seed, start, form == SV_MONTGOMERY ? 1 : 0);
  SV_HIP(hipGetLastError());
  SV_HIP(hipStreamSynchronize(st));
  return SV_OK;
}

int gen_bases_device(void* d, size_t n, uint64_t seed, uint64_t start, int form, int device,
                     hipStream_t user_stream) {
  if (n == 0) return SV_OK;
  WsLease lease(device, user_stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  hipStream_t st = lease.get()->stream;
  hipLaunchKernelGGL(k_gen_bases, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<G1Aff*>(d), (uint32_t)n, seed, start, form == SV_MONTGOMERY ? 1 : 0);
  SV_HIP(hipGetLastError());
  SV_HIP(hipStreamSynchronize(st));
  return SV_OK;
}

int powers_device(const void* d_r, int r_form, size_t n, int form_out, void* d_out, hipStream_t st) {
  hipLaunchKernelGGL(k_powers, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const Fr*>(d_r), r_form == SV_MONTGOMERY ? 1 : 0, (uint32_t)n,
                     form_out == SV_MONTGOMERY ? 1 : 0, reinterpret_cast<Fr*>(d_out));
  SV_HIP(hipGetLastError());
  return SV_OK;
}

}  // namespace sv
