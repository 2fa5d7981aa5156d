// f3 / f4: the data formats on either side of the path, decoded on the device.
//   k_decode_compressed  halo2curves' 32-byte compressed G1 (x LE, y parity in bit 255) -- what
//                        PoseidonTranscript::read_ec_point parses (system/halo2/transcript/
//                        halo2.rs:247-260): one square root (x^3 + 3)^((p+1)/4) per point
//   k_decode_evm         64-byte big-endian x || y (EvmTranscript::read_ec_point,
//                        transcript/evm.rs:223-242; also the G1 words of an EIP-197 record)
//   k_limbs_to_points    LimbsEncoding<LIMBS, BITS>::from_repr (pcs/kzg/accumulator.rs:57-77):
//                        fe_from_limbs (util/arithmetic.rs:262-274) + C::from_xy
// Every thread validates what the reference validates (canonical coordinates, on-curve, a square
// root exists) and records the first invalid index with atomicMin.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>

#include "codec.hpp"
#include "curve.hpp"
#include "runtime.hpp"

namespace sv {

namespace {

__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

__device__ __forceinline__ void put_point(G1Aff* out, const Fq& x, const Fq& y) {
  uint4* q = reinterpret_cast<uint4*>(out);
  q[0] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  q[1] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
  q[2] = make_uint4(y.v[0], y.v[1], y.v[2], y.v[3]);
  q[3] = make_uint4(y.v[4], y.v[5], y.v[6], y.v[7]);
}

// (x, y) canonical -> output in the requested form; identity (0, 0) stays (0, 0)
__device__ __forceinline__ void emit(G1Aff* out, Fq x, Fq y, int mont_out) {
  if (mont_out && !(x.is_zero() && y.is_zero())) {
    x = fe_to_mont(x);
    y = fe_to_mont(y);
  }
  put_point(out, x, y);
}

// y^2 == x^3 + 3 for canonical x, y
__device__ __forceinline__ bool on_curve(const Fq& x, const Fq& y) {
  const Fq xm = fe_to_mont(x), ym = fe_to_mont(y);
  return fe_sqr(ym) == fe_sqr(xm) * xm + fq_const(FQ_B3);
}

__global__ void k_decode_compressed(const uint8_t* __restrict__ in, uint32_t n, int mont_out, G1Aff* __restrict__ out,
                                    int* __restrict__ bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(in + (size_t)i * 32);
  Fq x;
#pragma unroll
  for (int k = 0; k < 8; k++) x.v[k] = w[k];
  const uint32_t sign = x.v[7] >> 31;
  x.v[7] &= 0x7fffffffu;
  if (!x.is_reduced()) {
    atomicMin(bad, (int)i);
    put_point(out + i, Fq::zero(), Fq::zero());
    return;
  }
  if (x.is_zero() && !sign) {  // identity
    put_point(out + i, Fq::zero(), Fq::zero());
    return;
  }
  const Fq xm = fe_to_mont(x);
  const Fq rhs = fe_sqr(xm) * xm + fq_const(FQ_B3);
  Fq y = Fq::one();
  for (int li = 7; li >= 0; li--)
    for (int b = 31; b >= 0; b--) {
      y = fe_sqr_hp(y);
      if ((FQ_SQRT_EXP[li] >> b) & 1) y = y * rhs;
    }
  if (fe_sqr(y) != rhs) {
    atomicMin(bad, (int)i);
    put_point(out + i, Fq::zero(), Fq::zero());
    return;
  }
  Fq yc = fe_from_mont(y);
  if ((yc.v[0] & 1u) != sign) {
    y = -y;
    yc = fe_from_mont(y);
  }
  put_point(out + i, mont_out ? xm : x, mont_out ? y : yc);
}

// record i starts at in + i * stride + offset: 32-byte BE x, then 32-byte BE y
__global__ void k_decode_evm(const uint8_t* __restrict__ in, uint32_t n, uint32_t stride, uint32_t offset,
                             int mont_out, G1Aff* __restrict__ out, int* __restrict__ bad) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* r = in + (size_t)i * stride + offset;
  Fq x, y;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t a, b;
    memcpy(&a, r + 28 - 4 * k, 4);  // records may be unaligned (EIP-197 words sit at 32-byte steps)
    memcpy(&b, r + 60 - 4 * k, 4);
    x.v[k] = bswap32(a);
    y.v[k] = bswap32(b);
  }
  const bool ident = x.is_zero() && y.is_zero();
  if (!x.is_reduced() || !y.is_reduced() || (!ident && !on_curve(x, y))) {
    atomicMin(bad, (int)i);
    put_point(out + i, Fq::zero(), Fq::zero());
    return;
  }
  emit(out + i, x, y, mont_out);
}

// point p: limbs [2pL, 2pL + L) -> x, [2pL + L, 2pL + 2L) -> y; out_even / out_odd by p's parity
// (an accumulator is lhs = point 2j, rhs = point 2j + 1)
__global__ void k_limbs_to_points(const Fr* __restrict__ limbs, uint32_t npts, int L, int bits, int mont_in,
                                  int mont_out, G1Aff* __restrict__ out_even, G1Aff* __restrict__ out_odd,
                                  int* __restrict__ bad) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npts) return;
  Fq c[2];
  bool ok = true;
  for (int j = 0; j < 2; j++) {
    uint32_t acc[17];
#pragma unroll
    for (int k = 0; k < 17; k++) acc[k] = 0;
    for (int i = 0; i < L; i++) {
      const uint32_t* lp = reinterpret_cast<const uint32_t*>(limbs + ((size_t)p * 2 + j) * L + i);
      Fr lv;
#pragma unroll
      for (int k = 0; k < 8; k++) lv.v[k] = lp[k];
      if (!lv.is_reduced()) ok = false;  // limbs are Fr elements
      if (mont_in) lv = fe_from_mont(lv);
      const int sh = bits * i, sw = sh >> 5, sb = sh & 31;
      uint64_t carry = 0;
      for (int k = 0; k + sw < 17; k++) {
        const uint64_t lo = k < 8 ? lv.v[k] : 0u;
        const uint64_t hi = (k >= 1 && k - 1 < 8) ? lv.v[k - 1] : 0u;
        const uint32_t part = sb ? (uint32_t)((lo << sb) | (hi >> (32 - sb))) : (uint32_t)lo;
        const uint64_t s = (uint64_t)acc[k + sw] + part + carry;
        acc[k + sw] = (uint32_t)s;
        carry = s >> 32;
      }
    }
    // fe_from_big: at most 32 bytes, and from_repr: < p
    for (int k = 8; k < 17; k++)
      if (acc[k]) ok = false;
#pragma unroll
    for (int k = 0; k < 8; k++) c[j].v[k] = acc[k];
    if (!c[j].is_reduced()) ok = false;
  }
  G1Aff* o = (p & 1 ? out_odd : out_even) + (p >> 1);
  const bool ident = c[0].is_zero() && c[1].is_zero();
  if (!ok || (!ident && !on_curve(c[0], c[1]))) {
    atomicMin(bad, (int)(p >> 1));
    put_point(o, Fq::zero(), Fq::zero());
    return;
  }
  emit(o, c[0], c[1], mont_out);
}

int bad_begin(Workspace* ws, int** d_bad) {
  SV_TRY(ws->reserve(256));
  SV_TRY(ws->reserve_pinned(256));
  *d_bad = ws->carve<int>(1);
  SV_HIP(hipMemsetAsync(*d_bad, 0x7f, 4, ws->stream));  // 0x7f7f7f7f: above any index
  return SV_OK;
}

int bad_end(Workspace* ws, int* d_bad, int64_t* first_invalid) {
  SV_HIP(hipGetLastError());
  SV_HIP(hipMemcpyAsync(ws->pinned, d_bad, 4, hipMemcpyDeviceToHost, ws->stream));
  SV_HIP(hipStreamSynchronize(ws->stream));
  int b;
  memcpy(&b, ws->pinned, 4);
  *first_invalid = b == 0x7f7f7f7f ? -1 : b;
  return SV_OK;
}

}  // namespace

int g1_decode_device(const void* d_data, size_t n, int encoding, size_t stride, size_t offset, int form, int device,
                     hipStream_t stream, void* d_out, int64_t* first_invalid) {
  *first_invalid = -1;
  if (n == 0) return SV_OK;
  if (n >= 0x7f000000ull) return SV_ERR_LEN;  // indices stay below the 0x7f7f7f7f sentinel
  WsLease lease(device, stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  int* bad;
  SV_TRY(bad_begin(ws, &bad));
  const uint32_t blocks = (uint32_t)((n + 255) / 256);
  const int mont = form == SV_MONTGOMERY;
  const uint8_t* in = static_cast<const uint8_t*>(d_data);
  G1Aff* out = static_cast<G1Aff*>(d_out);
  if (encoding == SV_ENC_HALO2_COMPRESSED) {
    hipLaunchKernelGGL(k_decode_compressed, dim3(blocks), dim3(256), 0, ws->stream, in, (uint32_t)n, mont, out, bad);
  } else if (encoding == SV_ENC_EVM) {
    hipLaunchKernelGGL(k_decode_evm, dim3(blocks), dim3(256), 0, ws->stream, in, (uint32_t)n,
                       (uint32_t)(stride ? stride : 64), (uint32_t)offset, mont, out, bad);
  } else {
    set_error("unknown point encoding %d", encoding);
    return SV_ERR_ARG;
  }
  return bad_end(ws, bad, first_invalid);
}

int limbs_to_accumulators_device(const void* d_limbs, size_t n, int n_limbs, int bits, int form, int device,
                                 hipStream_t stream, void* d_lhs, void* d_rhs, int64_t* first_invalid) {
  *first_invalid = -1;
  if (n == 0) return SV_OK;
  if (n >= 0x3f000000ull) return SV_ERR_LEN;
  if (n_limbs < 1 || bits < 1 || bits > 256 || (int64_t)bits * (n_limbs - 1) > 255) {
    set_error("limb codec: LIMBS = %d, BITS = %d out of range", n_limbs, bits);
    return SV_ERR_ARG;
  }
  WsLease lease(device, stream);
  if (!lease.ok()) return SV_ERR_DEVICE;
  Workspace* ws = lease.get();
  int* bad;
  SV_TRY(bad_begin(ws, &bad));
  const uint32_t npts = (uint32_t)(2 * n);
  const int mont = form == SV_MONTGOMERY;
  hipLaunchKernelGGL(k_limbs_to_points, dim3((npts + 255) / 256), dim3(256), 0, ws->stream,
                     static_cast<const Fr*>(d_limbs), npts, n_limbs, bits, mont, mont, static_cast<G1Aff*>(d_lhs),
                     static_cast<G1Aff*>(d_rhs), bad);
  return bad_end(ws, bad, first_invalid);
}

}  // namespace sv
