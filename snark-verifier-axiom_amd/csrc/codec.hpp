// Device decoders for the data formats around the path (see codec.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/svgpu.h"

namespace sv {
// n points; EVM records are read at d_data + i * stride + offset (stride 0 = 64).  Output affine
// in `form`, invalid points written as (0, 0); *first_invalid = lowest invalid index or -1.
// Synchronous on `stream`.
int g1_decode_device(const void* d_data, size_t n, int encoding, size_t stride, size_t offset, int form, int device,
                     hipStream_t stream, void* d_out, int64_t* first_invalid);
// n accumulators of 4 * n_limbs Fr limbs each -> lhs[i], rhs[i]; *first_invalid = lowest invalid
// accumulator or -1.  `form` applies to the limbs and to the output points.
int limbs_to_accumulators_device(const void* d_limbs, size_t n, int n_limbs, int bits, int form, int device,
                                 hipStream_t stream, void* d_lhs, void* d_rhs, int64_t* first_invalid);
}  // namespace sv
