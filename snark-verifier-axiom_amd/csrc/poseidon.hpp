#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace sv {
// In-place x^5 Poseidon permutation of n states of t Fr elements (t = 3 or 5), device buffers.
int poseidon_permute_device(void* d_states, size_t n, int t, int form, hipStream_t st);
// Poseidon::squeeze on n sponges: states (n x t, in/out) absorb d_elements[off[j] .. off[j+1])
// (d_offsets has n + 1 entries) and are squeezed; d_out[j] = state[1] (d_out may be null).
int poseidon_squeeze_device(void* d_states, const void* d_elements, const uint64_t* d_offsets, size_t n, int t,
                           int form, void* d_out, hipStream_t st);
}  // namespace sv
