#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace sv {
int gen_scalars_device(void* d, size_t n, uint64_t seed, uint64_t start, int form, int device,
                       hipStream_t stream);
int gen_bases_device(void* d, size_t n, uint64_t seed, uint64_t start, int form, int device,
                     hipStream_t stream);
// d_out[i] = r^i for i < n (r on the device in form r_form; output in form_out).
int powers_device(const void* d_r, int r_form, size_t n, int form_out, void* d_out, hipStream_t st);
}  // namespace sv
