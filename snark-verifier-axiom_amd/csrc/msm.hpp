// Pippenger MSM plan + entry points (see msm.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <vector>

#include "../../include/svgpu.h"
#include "host_ec.hpp"

namespace sv {

struct MsmPlan {
  int c;            // window bits (signed digits: 2^(c-1) buckets per window)
  uint32_t W;       // windows = ceil(255 / c)
  uint32_t B;       // buckets per window
  uint32_t nbt;     // W * B
  uint32_t K;       // sorted entries per accumulate thread
  uint32_t T;       // accumulate threads
  uint32_t logL;    // log2 of the buckets per running-sum segment
  uint32_t J;       // running-sum segments per window (B >> logL)
  uint32_t logJ;    // log2(J)
  uint32_t NG;      // subset-sum groups per window: 2 + logJ
  bool glv;         // GLV split: 2n virtual points (P, phi(P)) with 128-bit scalar halves
  size_t npts;      // virtual points: n, or 2n with GLV
  int phi64;        // GLV table: whole phi(P) records (1) or beta x only (0)
  int tree;         // bucket reduction: 0 k_wsum + k_group_sum, 1 running sums + tree, 2 tree over buckets
  int r29;          // k_accumulate's chain: 29-bit limbs, sums stored as x R' words (1) or 32-bit (0)
};

MsmPlan msm_plan(size_t n);

// MSMs of at most this many terms skip the pipeline: window sums on the device, the window Horner on
// the host (msm_batch_windows_host); SVGPU_SMALL_MSM=0 keeps the pipeline for them.
constexpr size_t kSmallMsmTerms = 256;

// Device-resident MSM on `device`; result (XYZZ, Montgomery) on the host.
int msm_run_device(const void* d_bases, const void* d_scalars, size_t n, int form, int device,
                   hipStream_t stream, host::Xyzz* out);

// Host-fed MSM (the host-buffer entry points): the caller's inputs reach HBM in `pieces` pieces on
// the workspace's copy stream.  stage_scalars(lo, hi, d_scalars, copy_stream, ready) and
// stage_bases(lo, hi, d_bases, copy_stream, ready) issue the transfers of points [lo, hi) into the
// given device pointers and record `ready` after them.  They are called in that order per piece,
// with the piece's sort enqueued in between: pageable transfers block the calling thread, so the
// sort then runs while the bases are still in flight.
struct MsmFeed {
  int pieces = 0;             // equal pieces (0: split, else the default schedule)
  std::vector<double> split;  // piece weights from 2^18 points when SVGPU_H2D_* are unset

  std::function<int(size_t lo, size_t hi, void* d_scalars, hipStream_t copy_stream, hipEvent_t ready)> stage_scalars;
  std::function<int(size_t lo, size_t hi, void* d_bases, hipStream_t copy_stream, hipEvent_t ready)> stage_bases;
};
int msm_run_fed(size_t n, int form, int device, const MsmFeed& feed, host::Xyzz* out);

int msm_last_stats(sv_msm_stats* out);

}  // namespace sv
