// Batched small MSMs (see msm_batch.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace sv {
// count MSMs; MSM k = sum over i in [off[k], off[k+1]) of scalars[i] * bases[i] (device arrays);
// d_out[k] = affine result in `form`.  max_terms (the largest MSM) only picks the window size.
// d_ids (optional): launch only MSMs d_ids[0..count) (results still land at d_out[id]).
// d_bidx (optional): base table mode -- term i uses d_bases[d_bidx[i]] (indices < table_len, else
// SV_ERR_ARG), the table in `base_form`; scalars and outputs stay in `form`.
// Synchronous on `stream`.
int msm_batch_device(const void* d_bases, const void* d_scalars, const uint64_t* d_offsets, const uint32_t* d_ids,
                     size_t count, size_t max_terms, int form, int device, hipStream_t stream, void* d_out,
                     const uint32_t* d_bidx = nullptr, uint64_t table_len = 0, int base_form = 0);
int msm_batch_window_bits(size_t max_terms);
// A few small MSMs (each at most 256 terms, the largest max_terms) with the window sums on the device
// and the window Horner on the host: out[k] = MSM k as a host XYZZ point (Montgomery).  Scalars in
// scalar_form, bases in base_form.  Synchronous on `stream`.
namespace host { struct Xyzz; }
int msm_batch_windows_host(const void* d_bases, const void* d_scalars, const uint64_t* d_offsets, size_t count,
                           size_t max_terms, int scalar_form, int base_form, int device, hipStream_t stream,
                           host::Xyzz* out);

// Precomputed base tables: every row P expanded to its window multiples 2^(8 w) P (affine,
// Montgomery) so that table-backed MSMs need one bucket set and no window Horner.
size_t table_precomputed_rows_bytes(size_t n);
int table_precompute_device(const void* d_rows, size_t n, void* d_pre, int device);
// MSM k = sum over i in [off[k], off[k+1]) of scalars[i] * table[bidx[i]] from the precomputed rows;
// an empty MSM gives the identity; index >= rows or an unreduced scalar is SV_ERR_ARG.  Synchronous.
int msm_batch_fixed_device(const void* d_pre, size_t rows, const uint32_t* d_bidx, const void* d_scalars,
                           const uint64_t* d_offsets, size_t count, int form, int device, hipStream_t stream,
                           void* d_out);
}  // namespace sv
