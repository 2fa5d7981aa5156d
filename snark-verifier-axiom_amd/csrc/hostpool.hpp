// Host worker pool shared by every libsvgpu call (no HIP dependency: the ThreadSanitizer stress
// test in tests/native builds this file alone).  SVGPU_HOST_THREADS, default min(16, cores).
#pragma once
#include <cstddef>
#include <functional>

namespace sv {

// fn(lo, hi) over contiguous slices of [0, n) of at least `grain` items, run on the pool and the
// caller; returns once every slice has run.  Concurrent callers are serialised (one job at a time).
void host_parallel_for(size_t n, size_t grain, const std::function<void(size_t, size_t)>& fn);
int host_threads();

}  // namespace sv
