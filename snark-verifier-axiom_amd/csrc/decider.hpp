#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/svgpu.h"

namespace sv {

int decide_run_device(const sv_g2_affine* g2, const sv_g2_affine* s_g2, const void* d_lhs,
                      const void* d_rhs, size_t n, int form, int device, hipStream_t stream,
                      int32_t* first_fail, int32_t* verdicts_host, sv_fq12* gt_host);

float& decider_last_kernel_ms();

}  // namespace sv
