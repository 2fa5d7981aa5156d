// FETCH_SIZE calibration for k_accumulate's access pattern (MI355X_MICROARCH.md HBM note: only
// 16-B/lane streaming reads are calibrated; other patterns must be calibrated on a known byte
// count).  k_gather64: every lane gathers random 64-B records (4 x 16-B loads, as load_aff does)
// from a table -- 64 MiB (the 2^20-point base table) and 1 GiB (larger than the 256 MiB Infinity
// Cache) -- k_stream: 16-B/lane coalesced streaming reads (the guide's calibrated case).  Run under
// rocprofv3 --pmc FETCH_SIZE; the known byte counts are printed.
// Build: hipcc -O3 --offload-arch=gfx950 tools/calib_fetch.hip -o tools/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void k_gather64(const uint4* __restrict__ tab, uint64_t nrec, uint32_t per_lane, uint32_t seed,
                           uint4* __restrict__ sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x = t * 2654435761u + seed;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint32_t k = 0; k < per_lane; k++) {
    x = x * 1664525u + 1013904223u;
    const uint64_t r = ((uint64_t)x * nrec) >> 32;
    const uint4* p = tab + r * 4;
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    acc.x ^= a.x ^ b.y ^ c.z ^ d.w;
    acc.y += a.y + b.x + c.w + d.z;
  }
  if (acc.x == 0x12345678u) sink[t] = acc;
}

__global__ void k_stream(const uint4* __restrict__ src, uint64_t n16, uint4* __restrict__ sink) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = src[i];
    acc.x ^= v.x;
    acc.y += v.y;
  }
  if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}

int main() {
  const size_t big = (size_t)1 << 30;
  uint4* tab;
  uint4* sink;
  if (hipMalloc(&tab, big) != hipSuccess || hipMalloc(&sink, 64 << 20) != hipSuccess) return 1;
  (void)hipMemset(tab, 1, big);
  const uint32_t threads = 1 << 20, per_lane = 16;
  for (size_t tbytes : {(size_t)64 << 20, big}) {
    const uint64_t nrec = tbytes / 64;
    hipLaunchKernelGGL(k_gather64, dim3(threads / 256), dim3(256), 0, 0, tab, nrec, per_lane, 7u, sink);
    (void)hipDeviceSynchronize();
    printf("k_gather64 table %zu MiB: known bytes %.1f MB (%u lanes x %u records x 64 B)\n", tbytes >> 20,
           (double)threads * per_lane * 64 / 1e6, threads, per_lane);
  }
  const uint64_t n16 = ((size_t)256 << 20) / 16;
  hipLaunchKernelGGL(k_stream, dim3(4096), dim3(256), 0, 0, tab, n16, sink);
  (void)hipDeviceSynchronize();
  printf("k_stream: known bytes %.1f MB\n", (double)n16 * 16 / 1e6);
  return 0;
}
