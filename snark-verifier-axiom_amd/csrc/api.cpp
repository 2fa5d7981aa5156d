// C ABI of libsvgpu (include/svgpu.h).  Every entry point is noexcept and maps failures to
// sv_status codes with a thread-local message (sv_last_error).  No CPU fallback: compute entry
// points need a GPU and return SV_ERR_DEVICE without one.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <mutex>
#include <unordered_map>
#include <string>
#include <thread>
#include <vector>

#include "../../include/svgpu.h"
#include "codec.hpp"
#include "decider.hpp"
#include "gen.hpp"
#include "host_ec.hpp"
#include "host_poseidon.hpp"
#include "msm.hpp"
#include "msm_batch.hpp"
#include "poseidon.hpp"
#include "runtime.hpp"

using namespace sv;
using sv::host::F;
using sv::host::Xyzz;

namespace {

F fe_in(const sv_fe& a) {
  F r;
  memcpy(r.l, a.l, 32);
  return r;
}
sv_fe fe_out(const F& a) {
  sv_fe r;
  memcpy(r.l, a.l, 32);
  return r;
}

void affine_out(const Xyzz& p, int form, sv_g1_affine* out) {
  F x, y;
  host::x_to_affine(p, x, y);
  if (form == SV_CANONICAL && !host::x_is_identity(p)) {
    x = host::f_from_mont(x);
    y = host::f_from_mont(y);
  }
  out->x = fe_out(x);
  out->y = fe_out(y);
}

void jacobian_out(const Xyzz& p, sv_g1_jacobian* out) {
  F X, Y, Z;
  host::x_to_jacobian(p, X, Y, Z);
  out->x = fe_out(host::f_from_mont(X));
  out->y = fe_out(host::f_from_mont(Y));
  out->z = fe_out(host::f_from_mont(Z));
}

int resolve_gpus(int num_gpus) {
  int have = runtime_device_count();
  if (have == 0) {
    if (runtime_init(0) != SV_OK) return 0;
    have = runtime_device_count();
  }
  if (num_gpus <= 0 || num_gpus > have) return have;
  return num_gpus;
}

// Runs fn(shard_index, device) on one host thread per device; returns the first non-OK status.
template <class Fn>
int for_each_device(int ndev, Fn fn) {
  std::vector<int> rc(ndev, SV_OK);
  std::vector<std::string> msg(ndev);
  if (ndev == 1) return fn(0, runtime_device_id(0));
  std::vector<std::thread> th;
  for (int d = 0; d < ndev; d++)
    th.emplace_back([&, d] {
      rc[d] = fn(d, runtime_device_id(d));
      if (rc[d] != SV_OK) msg[d] = sv::last_error();
    });
  for (auto& t : th) t.join();
  for (int d = 0; d < ndev; d++)
    if (rc[d] != SV_OK) {
      sv::set_error("device %d: %s", d, msg[d].c_str());
      return rc[d];
    }
  return SV_OK;
}

// Pooled device staging for the host-buffer entry points: the regions live in a leased
// workspace's grow-only input buffer (no per-call hipMalloc / hipFree); copies run on the lease's
// stream and are synchronised before the call returns.
struct Staging {
  WsLease lease;
  std::vector<char*> d;
  bool pending = false;  // async copies queued since the last sync (they may read caller memory)
  explicit Staging(int device) : lease(device, nullptr) {}
  Staging(const Staging&) = delete;
  Staging& operator=(const Staging&) = delete;
  // An early error return must not hand the workspace back to the pool (or free the host memory
  // a queued copy reads) while copies are still in flight.
  ~Staging() {
    if (pending && lease.ok()) (void)hipStreamSynchronize(lease.get()->stream);
  }
  int init(std::initializer_list<size_t> sizes) {
    if (!lease.ok()) return SV_ERR_DEVICE;
    size_t tot = 0;
    for (size_t s : sizes) tot += Workspace::aligned(s ? s : 1);
    SV_TRY(lease.get()->reserve_in(tot));
    char* p = lease.get()->inbuf;
    for (size_t s : sizes) {
      d.push_back(p);
      p += Workspace::aligned(s ? s : 1);
    }
    return SV_OK;
  }
  template <class T = void>
  T* at(int i) const {
    return reinterpret_cast<T*>(d[i]);
  }
  int put(int i, const void* h, size_t bytes) {
    pending = true;
    if (bytes) SV_HIP(hipMemcpyAsync(d[i], h, bytes, hipMemcpyHostToDevice, lease.get()->stream));
    return SV_OK;
  }
  int put_at(int i, size_t offset, const void* h, size_t bytes) {
    pending = true;
    if (bytes) SV_HIP(hipMemcpyAsync(d[i] + offset, h, bytes, hipMemcpyHostToDevice, lease.get()->stream));
    return SV_OK;
  }
  int get(void* h, int i, size_t bytes) {
    pending = true;
    if (bytes) SV_HIP(hipMemcpyAsync(h, d[i], bytes, hipMemcpyDeviceToHost, lease.get()->stream));
    return SV_OK;
  }
  int sync() {
    SV_HIP(hipStreamSynchronize(lease.get()->stream));
    pending = false;
    return SV_OK;
  }
};

// Small MSMs (at most kSmallMsmTerms terms each, msm.hpp) go through msm_batch_windows_host: window
// sums on the device, the window Horner on the host.  SVGPU_SMALL_MSM=0 keeps the single-MSM
// pipeline (read per call; results identical).
bool small_msm_off() {
  const char* e = getenv("SVGPU_SMALL_MSM");
  return e && atoi(e) == 0;
}

// pieces of a host-fed MSM (SVGPU_H2D_PIECES; unset = 0: the MSM plan picks, see msm_run_impl):
// piece k + 1's transfer overlaps piece k's sort and accumulation
int h2d_pieces() {
  const char* e = getenv("SVGPU_H2D_PIECES");
  if (!e) return 0;
  const int p = atoi(e);
  return p < 1 ? 1 : p;
}

#define SV_GUARD_BEGIN try {
#define SV_GUARD_END                                    \
  }                                                     \
  catch (const std::exception& e) {                     \
    sv::set_error("internal error: %s", e.what());      \
    return SV_ERR_DEVICE;                               \
  }                                                     \
  catch (...) {                                         \
    sv::set_error("internal error");                    \
    return SV_ERR_DEVICE;                               \
  }

int check_form(int form) {
  if (form != SV_CANONICAL && form != SV_MONTGOMERY) {
    sv::set_error("bad form %d", form);
    return SV_ERR_ARG;
  }
  return SV_OK;
}

}  // namespace

extern "C" {

int sv_init(int num_devices) noexcept {
  SV_GUARD_BEGIN
  return runtime_init(num_devices);
  SV_GUARD_END
}

int sv_device_count(void) noexcept {
  SV_GUARD_BEGIN
  return runtime_device_count();
  SV_GUARD_END
}

const char* sv_last_error(void) noexcept { return sv::last_error(); }

const char* sv_version(void) noexcept { return "svgpu 0.1.0 (abi 1, gfx950)"; }

int sv_bn254_g1_msm(const sv_g1_affine* bases, const sv_fe* scalars, size_t n, int form, int num_gpus,
                    sv_g1_affine* out) noexcept {
  SV_GUARD_BEGIN
  if (n == 0) {
    sv::set_error("pairs should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!bases || !scalars || !out) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  int ndev = resolve_gpus(num_gpus);
  if (ndev == 0) return SV_ERR_DEVICE;
  if ((size_t)ndev > n) ndev = (int)n;
  std::vector<Xyzz> part(ndev, host::x_identity());
  size_t per = (n + ndev - 1) / ndev;
  int rc = for_each_device(ndev, [&](int k, int dev) -> int {
    size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo >= hi) return SV_OK;
    MsmFeed feed;
    feed.pieces = h2d_pieces();
    // pageable caller memory: the runtime's staged DMA measured at the pinned rate (tools/ubench_h2d.cpp)
    feed.stage_scalars = [&, lo](size_t a, size_t b, void* ds, hipStream_t cs, hipEvent_t ready) -> int {
      SV_HIP(hipMemcpyAsync(ds, scalars + lo + a, (b - a) * sizeof(sv_fe), hipMemcpyHostToDevice, cs));
      SV_HIP(hipEventRecord(ready, cs));
      return SV_OK;
    };
    feed.stage_bases = [&, lo](size_t a, size_t b, void* db, hipStream_t cs, hipEvent_t ready) -> int {
      SV_HIP(hipMemcpyAsync(db, bases + lo + a, (b - a) * sizeof(sv_g1_affine), hipMemcpyHostToDevice, cs));
      SV_HIP(hipEventRecord(ready, cs));
      return SV_OK;
    };
    return msm_run_fed(hi - lo, form, dev, feed, &part[k]);
  });
  if (rc != SV_OK) return rc;
  Xyzz acc = host::x_identity();
  for (auto& p : part) acc = host::x_add(acc, p);
  affine_out(acc, form, out);
  return SV_OK;
  SV_GUARD_END
}

// references gathered this far ahead are prefetched (random 32/64-B reads are DRAM-latency bound);
// SVGPU_GATHER_AHEAD overrides (read once)
static size_t gather_ahead() {
  static const size_t a = getenv("SVGPU_GATHER_AHEAD") ? (size_t)std::max(1, atoi(getenv("SVGPU_GATHER_AHEAD"))) : 16;
  return a;
}

int sv_bn254_g1_msm_refs(const sv_msm_ref* pairs, size_t n, int form, int num_gpus, sv_g1_affine* out) noexcept {
  SV_GUARD_BEGIN
  if (n == 0) {
    sv::set_error("pairs should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!pairs || !out) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  int ndev = resolve_gpus(num_gpus);
  if (ndev == 0) return SV_ERR_DEVICE;
  if ((size_t)ndev > n) ndev = (int)n;
  std::vector<Xyzz> part(ndev, host::x_identity());
  size_t per = (n + ndev - 1) / ndev;
  int rc = for_each_device(ndev, [&](int k, int dev) -> int {
    size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo >= hi) return SV_OK;
    const size_t m = hi - lo;
    // the gather target: pinned staging of a leased workspace (grow-only, reused across calls)
    WsLease st_lease(dev, nullptr);
    if (!st_lease.ok()) return SV_ERR_DEVICE;
    Workspace* sw = st_lease.get();
    SV_TRY(sw->reserve_stage(m * (sizeof(sv_fe) + sizeof(sv_g1_affine))));
    sv_fe* hs = reinterpret_cast<sv_fe*>(sw->stage);
    sv_g1_affine* hb = reinterpret_cast<sv_g1_affine*>(sw->stage + m * sizeof(sv_fe));
    std::atomic<int> null_ref{0};
    MsmFeed feed;
    feed.pieces = h2d_pieces();
    // the gather paces this path: smaller first and middle pieces keep the gather, the DMA and the
    // accumulates overlapped (2^20: 2,2,3,3,3,3 3.67-3.73 ms, 4 equal pieces 3.95)
    feed.split = {2, 2, 3, 3, 3, 3};
    // gather piece [a, b) on the host pool (scalars, then bases: the scalar DMA and the piece's
    // sort overlap the base gather, and this piece's DMA the next piece's gather).  (Gathering both
    // in one pass per piece was measured slower: 3.7 -> 4.2-4.9 ms at 2^20, the sort then waits for
    // the whole piece.)
    const size_t kGatherAhead = gather_ahead();
    feed.stage_scalars = [&, lo](size_t a, size_t b, void* ds, hipStream_t cs, hipEvent_t ready) -> int {
      host_parallel_for(b - a, 8192, [&](size_t x, size_t y) {
        for (size_t i = a + x; i < a + y; i++) {
          if (i + kGatherAhead < a + y) __builtin_prefetch(pairs[lo + i + kGatherAhead].scalar);
          const sv_fe* sp = pairs[lo + i].scalar;
          if (!sp) {
            null_ref.store(1, std::memory_order_relaxed);
            memset(&hs[i], 0, sizeof(sv_fe));
          } else {
            hs[i] = *sp;
          }
        }
      });
      SV_HIP(hipMemcpyAsync(ds, hs + a, (b - a) * sizeof(sv_fe), hipMemcpyHostToDevice, cs));
      SV_HIP(hipEventRecord(ready, cs));
      return SV_OK;
    };
    feed.stage_bases = [&, lo](size_t a, size_t b, void* db, hipStream_t cs, hipEvent_t ready) -> int {
      host_parallel_for(b - a, 8192, [&](size_t x, size_t y) {
        for (size_t i = a + x; i < a + y; i++) {
          if (i + kGatherAhead < a + y) {
            const char* q = reinterpret_cast<const char*>(pairs[lo + i + kGatherAhead].base);
            __builtin_prefetch(q);
            __builtin_prefetch(q + 63);  // a 64-B point may straddle two lines
          }
          const sv_g1_affine* bp = pairs[lo + i].base;
          if (!bp) {
            null_ref.store(1, std::memory_order_relaxed);
            memset(&hb[i], 0, sizeof(sv_g1_affine));
          } else {
            hb[i] = *bp;
          }
        }
      });
      SV_HIP(hipMemcpyAsync(db, hb + a, (b - a) * sizeof(sv_g1_affine), hipMemcpyHostToDevice, cs));
      SV_HIP(hipEventRecord(ready, cs));
      return SV_OK;
    };
    int r = msm_run_fed(m, form, dev, feed, &part[k]);
    if (r == SV_OK && null_ref.load()) {
      sv::set_error("null scalar or base reference");
      return SV_ERR_ARG;
    }
    return r;
  });
  if (rc != SV_OK) return rc;
  Xyzz acc = host::x_identity();
  for (auto& p : part) acc = host::x_add(acc, p);
  affine_out(acc, form, out);
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_device(const sv_g1_affine* d_bases, const sv_fe* d_scalars, size_t n, int form,
                           int device, void* stream, sv_g1_jacobian* out_partial) noexcept {
  SV_GUARD_BEGIN
  if (n == 0) {
    sv::set_error("pairs should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!d_bases || !d_scalars || !out_partial) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  Xyzz r;
  SV_TRY(msm_run_device(d_bases, d_scalars, n, form, device, (hipStream_t)stream, &r));
  jacobian_out(r, out_partial);
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_fold(const sv_g1_jacobian* partials, size_t k, sv_g1_affine* out, int out_form) noexcept {
  SV_GUARD_BEGIN
  if (k == 0) {
    sv::set_error("no partials");
    return SV_ERR_EMPTY;
  }
  if (!partials || !out) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(out_form));
  Xyzz acc = host::x_identity();
  for (size_t i = 0; i < k; i++) {
    F X = fe_in(partials[i].x), Y = fe_in(partials[i].y), Z = fe_in(partials[i].z);
    if (!host::f_is_reduced(X) || !host::f_is_reduced(Y) || !host::f_is_reduced(Z)) {
      sv::set_error("partial %zu: coordinate not reduced", i);
      return SV_ERR_ARG;
    }
    acc = host::x_add(acc, host::x_from_jacobian(host::f_to_mont(X), host::f_to_mont(Y), host::f_to_mont(Z)));
  }
  affine_out(acc, out_form, out);
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_kzg_decide(const sv_g2_affine* g2, const sv_g2_affine* s_g2, const sv_g1_affine* lhs,
                        const sv_g1_affine* rhs, size_t n, int form, int num_gpus, int32_t* first_fail) noexcept {
  SV_GUARD_BEGIN
  if (n == 0) {
    sv::set_error("accumulators should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!g2 || !s_g2 || !lhs || !rhs || !first_fail) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  int ndev = resolve_gpus(num_gpus);
  if (ndev == 0) return SV_ERR_DEVICE;
  if ((size_t)ndev > n) ndev = (int)n;
  size_t per = (n + ndev - 1) / ndev;
  std::vector<int32_t> ff(ndev, -1);
  int rc = for_each_device(ndev, [&](int k, int dev) -> int {
    size_t lo = k * per, hi = std::min(n, lo + per);
    if (lo >= hi) return SV_OK;
    size_t m = hi - lo;
    Staging sg(dev);
    SV_TRY(sg.init({m * sizeof(sv_g1_affine), m * sizeof(sv_g1_affine)}));
    SV_TRY(sg.put(0, lhs + lo, m * sizeof(sv_g1_affine)));
    SV_TRY(sg.put(1, rhs + lo, m * sizeof(sv_g1_affine)));
    SV_TRY(sg.sync());
    int32_t f = -1;
    SV_TRY(decide_run_device(g2, s_g2, sg.at(0), sg.at(1), m, form, dev, nullptr, &f, nullptr, nullptr));
    ff[k] = f < 0 ? -1 : (int32_t)(lo + f);
    return SV_OK;
  });
  if (rc != SV_OK) return rc;
  *first_fail = -1;
  for (int k = 0; k < ndev; k++)
    if (ff[k] >= 0) {
      *first_fail = ff[k];
      break;
    }
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_kzg_decide_device(const sv_g2_affine* g2, const sv_g2_affine* s_g2, const sv_g1_affine* d_lhs,
                               const sv_g1_affine* d_rhs, size_t n, int form, int device, void* stream,
                               int32_t* first_fail, int32_t* verdicts, sv_fq12* gt) noexcept {
  SV_GUARD_BEGIN
  if (!g2 || !s_g2 || !d_lhs || !d_rhs) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  return decide_run_device(g2, s_g2, d_lhs, d_rhs, n, form, device, (hipStream_t)stream, first_fail,
                           verdicts, gt);
  SV_GUARD_END
}

int sv_bn254_kzg_accumulate(const sv_g1_affine* lhs, const sv_g1_affine* rhs, size_t n, const sv_fe* r,
                            int form, int num_gpus, sv_g1_affine* out_lhs, sv_g1_affine* out_rhs) noexcept {
  SV_GUARD_BEGIN
  (void)num_gpus;  // n is small (one scalar per accumulator): a single device suffices
  if (n == 0) {
    sv::set_error("accumulators should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!lhs || !rhs || !r || !out_lhs || !out_rhs) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  if (!host::f_is_reduced(fe_in(*r), host::R64)) {
    sv::set_error("r not reduced mod the scalar field order");
    return SV_ERR_ARG;
  }
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  int dev = runtime_device_id(0);
  if (n <= kSmallMsmTerms && !small_msm_off()) {
    // Round 5: the two MSMs as ONE small batch (msm_batch_windows_host): r^i on the host (n Fr
    // products, ~1 us; k_powers was a 28 us serial chain on one lane plus a synchronisation), the
    // window sums of both MSMs in one launch, the window Horner of both on the host.
    namespace fr = sv::host::fr;
    fr::E rm;
    memcpy(rm.l, r->l, 32);
    if (form != SV_MONTGOMERY) rm = fr::to_mont(rm);
    std::vector<sv_fe> pw(2 * n);
    fr::E acc = fr::one();
    for (size_t i = 0; i < n; i++) {
      memcpy(pw[i].l, acc.l, 32);
      pw[n + i] = pw[i];
      acc = fr::mul(acc, rm);
    }
    const uint64_t off[3] = {0, n, 2 * n};
    Staging sg(dev);
    SV_TRY(sg.init({2 * n * sizeof(sv_g1_affine), 2 * n * sizeof(sv_fe), sizeof off}));
    SV_TRY(sg.put(0, lhs, n * sizeof(sv_g1_affine)));
    SV_TRY(sg.put_at(0, n * sizeof(sv_g1_affine), rhs, n * sizeof(sv_g1_affine)));
    SV_TRY(sg.put(1, pw.data(), 2 * n * sizeof(sv_fe)));
    SV_TRY(sg.put(2, off, sizeof off));
    Xyzz ab[2];
    SV_TRY(msm_batch_windows_host(sg.at(0), sg.at(1), sg.at<const uint64_t>(2), 2, n, SV_MONTGOMERY, form, dev,
                                  sg.lease.get()->stream, ab));
    sg.pending = false;  // msm_batch_windows_host synchronised the stream
    affine_out(ab[0], form, out_lhs);
    affine_out(ab[1], form, out_rhs);
    return SV_OK;
  }
  Staging sg(dev);
  SV_TRY(sg.init({n * sizeof(sv_g1_affine), n * sizeof(sv_g1_affine), n * sizeof(sv_fe), sizeof(sv_fe)}));
  SV_TRY(sg.put(0, lhs, n * sizeof(sv_g1_affine)));
  SV_TRY(sg.put(1, rhs, n * sizeof(sv_g1_affine)));
  SV_TRY(sg.put(3, r, sizeof(sv_fe)));
  SV_TRY(sg.sync());
  SV_TRY(powers_device(sg.at(3), form, n, form, sg.at(2), sg.lease.get()->stream));
  SV_TRY(sg.sync());
  // the lhs and rhs MSMs share the scalars and are independent: run them concurrently (each call
  // leases its own stream + workspace), one on the caller and one on a pool worker
  Xyzz ab[2];
  int rc2[2] = {SV_OK, SV_OK};
  std::string err2[2];
  host_parallel_for(2, 1, [&](size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; k++) {
      rc2[k] = msm_run_device(sg.at(k == 0 ? 0 : 1), sg.at(2), n, form, dev, nullptr, &ab[k]);
      if (rc2[k] != SV_OK) err2[k] = sv::last_error();
    }
  });
  for (int k = 0; k < 2; k++)
    if (rc2[k] != SV_OK) {
      sv::set_error("%s", err2[k].c_str());
      return rc2[k];
    }
  const Xyzz& a = ab[0];
  const Xyzz& b = ab[1];
  affine_out(a, form, out_lhs);
  affine_out(b, form, out_rhs);
  return SV_OK;
  SV_GUARD_END
}

// KzgAs::create_proof without blind (accumulation.rs:146-195): a fresh PoseidonTranscript
// (T = 3, RATE = 2, R_F = 8, R_P = 57; snark-verifier-sdk/src/halo2.rs:52-55) absorbs every lhs_i,
// rhs_i through common_ec_point (transcript/halo2.rs:214-226: the affine x and y, each Fq -> Fr by
// fe_to_fe = reduction mod r) and squeezes r (:158-176); then the two r^i MSMs.  The sponge is one
// serial chain of n + 1 permutations and runs on the host (host_poseidon.hpp: a GPU lane would
// take ~20 ms for it at n = 64); the MSMs run on the device (sv_bn254_kzg_accumulate).
int sv_bn254_kzg_create_proof(const sv_g1_affine* lhs, const sv_g1_affine* rhs, size_t n, int form, int num_gpus,
                              sv_g1_affine* out_lhs, sv_g1_affine* out_rhs, sv_fe* sponge_state,
                              sv_fe* out_r) noexcept {
  SV_GUARD_BEGIN
  if (n == 0) {
    sv::set_error("accumulators should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!lhs || !rhs || !out_lhs || !out_rhs) {
    sv::set_error("null pointer");
    return SV_ERR_ARG;
  }
  SV_TRY(check_form(form));
  namespace fr = sv::host::fr;
  fr::Sponge3 sponge;
  if (sponge_state) {
    for (int k = 0; k < 3; k++) {
      fr::E e;
      memcpy(e.l, sponge_state[k].l, 32);
      if (!fr::is_reduced(e)) {
        sv::set_error("sponge_state[%d] not reduced mod r", k);
        return SV_ERR_ARG;
      }
      sponge.st[k] = form == SV_MONTGOMERY ? e : fr::to_mont(e);
    }
  }
  sponge.buf.reserve(4 * n);
  for (size_t i = 0; i < n; i++) {
    for (const sv_g1_affine* pt : {&lhs[i], &rhs[i]}) {
      F x = fe_in(pt->x), y = fe_in(pt->y);
      if (host::f_is_zero(x) && host::f_is_zero(y)) {
        // coordinates() of the identity is None -> Error::Transcript (halo2.rs:215-223)
        sv::set_error("Invalid elliptic curve point encoding in proof (accumulator %zu is the identity)", i);
        return SV_ERR_ARG;
      }
      if (!host::f_is_reduced(x) || !host::f_is_reduced(y)) {
        sv::set_error("accumulator %zu: coordinate not reduced mod p", i);
        return SV_ERR_ARG;
      }
      if (form == SV_MONTGOMERY) x = host::f_from_mont(x), y = host::f_from_mont(y);
      for (const F& c : {x, y}) {
        fr::E e;
        memcpy(e.l, c.l, 32);
        sponge.update(fr::to_mont(fr::reduce_below_2r(e)));  // fe_to_fe: canonical Fq mod r
      }
    }
  }
  const fr::E rm = sponge.squeeze();
  const fr::E rv = form == SV_MONTGOMERY ? rm : fr::from_mont(rm);
  sv_fe r;
  memcpy(r.l, rv.l, 32);
  const int rc = sv_bn254_kzg_accumulate(lhs, rhs, n, &r, form, num_gpus, out_lhs, out_rhs);
  if (rc != SV_OK) return rc;
  if (out_r) *out_r = r;
  if (sponge_state)
    for (int k = 0; k < 3; k++) {
      const fr::E e = form == SV_MONTGOMERY ? sponge.st[k] : fr::from_mont(sponge.st[k]);
      memcpy(sponge_state[k].l, e.l, 32);
    }
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_batch(const sv_g1_affine* bases, const sv_fe* scalars, const uint64_t* offsets, size_t count,
                          int form, sv_g1_affine* out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (count == 0) return SV_OK;
  if (!offsets || !out) return SV_ERR_ARG;
  for (size_t k = 0; k < count; k++) {
    if (offsets[k + 1] < offsets[k]) {
      sv::set_error("msm_batch: offsets not non-decreasing at %zu", k);
      return SV_ERR_ARG;
    }
    if (offsets[k + 1] == offsets[k]) {
      sv::set_error("pairs should not be empty (msm %zu)", k);
      return SV_ERR_EMPTY;
    }
  }
  if (!bases || !scalars) return SV_ERR_ARG;
  if (count > 0x7fffffffull) return SV_ERR_LEN;
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  size_t big_limit = 4096;
  if (const char* e = getenv("SVGPU_BATCH_MAX")) big_limit = strtoull(e, nullptr, 10);
  const uint64_t base = offsets[0], total = offsets[count] - base;
  std::vector<uint64_t> off(offsets, offsets + count + 1);
  for (auto& o : off) o -= base;
  // The fused batch kernel costs about one Horner chain (~0.65 ms) whatever the batch size, so in a
  // tiny batch (at most SVGPU_BATCH_SEQ_MAX MSMs) the MSMs above kSmallMsmTerms terms go through the
  // single-MSM pipeline one by one.  MSMs of at most kSmallMsmTerms terms stay in the batch: a batch
  // of only such MSMs passes no id map, so msm_batch_device can take its small-batch route (window
  // sums on the device, one host Horner per MSM: 0.17-0.20 ms for 1-16 MSMs of 64 terms).
  size_t seq_max = 4;
  if (const char* e = getenv("SVGPU_BATCH_SEQ_MAX")) seq_max = strtoull(e, nullptr, 10);
  if (count <= seq_max) big_limit = std::min(big_limit, kSmallMsmTerms);
  std::vector<uint32_t> small_ids, big_ids;
  size_t max_small = 0;
  for (size_t k = 0; k < count; k++) {
    const size_t m = off[k + 1] - off[k];
    if (m > big_limit) {
      big_ids.push_back((uint32_t)k);
    } else {
      small_ids.push_back((uint32_t)k);
      max_small = std::max(max_small, m);
    }
  }
  Staging sg(dev);
  SV_TRY(sg.init({total * sizeof(sv_g1_affine), total * sizeof(sv_fe), (count + 1) * sizeof(uint64_t),
                  count * sizeof(uint32_t), count * sizeof(sv_g1_affine)}));
  SV_TRY(sg.put(0, bases + base, total * sizeof(sv_g1_affine)));
  SV_TRY(sg.put(1, scalars + base, total * sizeof(sv_fe)));
  SV_TRY(sg.put(2, off.data(), (count + 1) * sizeof(uint64_t)));
  SV_TRY(sg.put(3, small_ids.data(), small_ids.size() * sizeof(uint32_t)));
  SV_TRY(sg.sync());
  if (!small_ids.empty()) {
    // every MSM small: no id map (the ids would be the identity), which the small-batch route needs
    const uint32_t* ids = big_ids.empty() ? nullptr : sg.at<const uint32_t>(3);
    SV_TRY(msm_batch_device(sg.at(0), sg.at(1), sg.at<const uint64_t>(2), ids, small_ids.size(), max_small, form, dev,
                            nullptr, sg.at(4)));
    SV_TRY(sg.get(out, 4, count * sizeof(sv_g1_affine)));
    SV_TRY(sg.sync());
  }
  for (uint32_t k : big_ids) {
    Xyzz r;
    SV_TRY(msm_run_device(sg.at<const sv_g1_affine>(0) + off[k], sg.at<const sv_fe>(1) + off[k],
                          off[k + 1] - off[k], form, dev, nullptr, &r));
    affine_out(r, form, &out[k]);
  }
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_batch_device(const sv_g1_affine* d_bases, const sv_fe* d_scalars, const uint64_t* d_offsets,
                                 size_t count, size_t max_terms, int form, int device, void* stream,
                                 sv_g1_affine* d_out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (count == 0) return SV_OK;
  if (!d_bases || !d_scalars || !d_offsets || !d_out) return SV_ERR_ARG;
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  SV_HIP(hipSetDevice(device));
  return msm_batch_device(d_bases, d_scalars, d_offsets, nullptr, count, max_terms, form, device, (hipStream_t)stream,
                          d_out);
  SV_GUARD_END
}

// ---- fixed-base tables (device-resident constant bases for batched MSMs) -------------------
namespace {
struct BaseTable {
  int dev = 0;
  void* p = nullptr;    // rows (Montgomery affine)
  void* pre = nullptr;  // rows expanded to their window multiples 2^(8 w) P (msm_batch_fixed_device)
  size_t n = 0;
};
std::mutex g_tables_mu;
std::unordered_map<uint64_t, BaseTable> g_tables;
uint64_t g_next_table = 1;

bool table_lookup(uint64_t h, BaseTable* out) {
  std::lock_guard<std::mutex> lk(g_tables_mu);
  auto it = g_tables.find(h);
  if (it == g_tables.end()) return false;
  *out = it->second;
  return true;
}

int check_offsets(const uint64_t* offsets, size_t count) {
  for (size_t k = 0; k < count; k++) {
    if (offsets[k + 1] < offsets[k]) {
      sv::set_error("msm_batch: offsets not non-decreasing at %zu", k);
      return SV_ERR_ARG;
    }
    if (offsets[k + 1] == offsets[k]) {
      sv::set_error("pairs should not be empty (msm %zu)", k);
      return SV_ERR_EMPTY;
    }
  }
  return SV_OK;
}
}  // namespace

int sv_bn254_g1_table_create(const sv_g1_affine* bases, size_t n, int form, int device, uint64_t* handle) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (!handle || (!bases && n)) return SV_ERR_ARG;
  if (n == 0) {
    sv::set_error("empty base table");
    return SV_ERR_EMPTY;
  }
  if (n > 0xffffffffull) return SV_ERR_LEN;
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  if (device < 0 || device >= runtime_device_count()) {
    sv::set_error("device %d not initialised", device);
    return SV_ERR_ARG;
  }
  const int dev = runtime_device_id(device);
  // Montgomery form on the device; coordinates must be reduced (as for every MSM input)
  std::vector<sv_g1_affine> mont(n);
  for (size_t i = 0; i < n; i++) {
    F x, y;
    memcpy(x.l, bases[i].x.l, 32);
    memcpy(y.l, bases[i].y.l, 32);
    if (!sv::host::f_is_reduced(x) || !sv::host::f_is_reduced(y)) {
      sv::set_error("base table row %zu: coordinate not reduced mod p", i);
      return SV_ERR_ARG;
    }
    const bool ident = sv::host::f_is_zero(x) && sv::host::f_is_zero(y);
    if (form == SV_CANONICAL && !ident) {
      x = sv::host::f_to_mont(x);
      y = sv::host::f_to_mont(y);
    }
    memcpy(mont[i].x.l, x.l, 32);
    memcpy(mont[i].y.l, y.l, 32);
  }
  BaseTable t;
  t.dev = dev;
  t.n = n;
  SV_HIP(hipSetDevice(dev));
  SV_HIP(hipMalloc(&t.p, n * sizeof(sv_g1_affine)));
  if (hipMalloc(&t.pre, table_precomputed_rows_bytes(n)) != hipSuccess) {
    (void)hipFree(t.p);
    sv::set_error("base table: precomputed rows hipMalloc failed");
    return SV_ERR_OOM;
  }
  int prc = hipMemcpy(t.p, mont.data(), n * sizeof(sv_g1_affine), hipMemcpyHostToDevice) == hipSuccess
                ? table_precompute_device(t.p, n, t.pre, dev)
                : SV_ERR_DEVICE;
  if (prc != SV_OK) {
    (void)hipFree(t.p);
    (void)hipFree(t.pre);
    sv::set_error("base table upload / precompute failed");
    return prc;
  }
  std::lock_guard<std::mutex> lk(g_tables_mu);
  *handle = g_next_table++;
  g_tables[*handle] = t;
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_table_destroy(uint64_t handle) noexcept {
  SV_GUARD_BEGIN
  BaseTable t;
  {
    std::lock_guard<std::mutex> lk(g_tables_mu);
    auto it = g_tables.find(handle);
    if (it == g_tables.end()) {
      sv::set_error("unknown base table handle %llu", (unsigned long long)handle);
      return SV_ERR_ARG;
    }
    t = it->second;
    g_tables.erase(it);
  }
  SV_HIP(hipSetDevice(t.dev));
  SV_HIP(hipFree(t.p));
  SV_HIP(hipFree(t.pre));
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_batch_table(uint64_t handle, const uint32_t* base_idx, const sv_fe* scalars,
                                const uint64_t* offsets, size_t count, int form, sv_g1_affine* out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (count == 0) return SV_OK;
  if (!offsets || !out) return SV_ERR_ARG;
  SV_TRY(check_offsets(offsets, count));
  if (!base_idx || !scalars) return SV_ERR_ARG;
  if (count > 0x7fffffffull) return SV_ERR_LEN;
  BaseTable t;
  if (!table_lookup(handle, &t)) {
    sv::set_error("unknown base table handle %llu", (unsigned long long)handle);
    return SV_ERR_ARG;
  }
  const uint64_t base = offsets[0], total = offsets[count] - base;
  size_t max_terms = 0;
  std::vector<uint64_t> off(offsets, offsets + count + 1);
  for (auto& o : off) o -= base;
  for (size_t k = 0; k < count; k++) max_terms = std::max<size_t>(max_terms, off[k + 1] - off[k]);
  for (uint64_t i = 0; i < total; i++)
    if (base_idx[base + i] >= t.n) {
      sv::set_error("msm_batch: base index %u at term %llu out of the table (%zu rows)", base_idx[base + i],
                    (unsigned long long)(base + i), t.n);
      return SV_ERR_ARG;
    }
  Staging sg(t.dev);
  SV_TRY(sg.init({total * sizeof(uint32_t), total * sizeof(sv_fe), (count + 1) * sizeof(uint64_t),
                  count * sizeof(sv_g1_affine)}));
  SV_TRY(sg.put(0, base_idx + base, total * sizeof(uint32_t)));
  SV_TRY(sg.put(1, scalars + base, total * sizeof(sv_fe)));
  SV_TRY(sg.put(2, off.data(), (count + 1) * sizeof(uint64_t)));
  SV_TRY(sg.sync());
  (void)max_terms;
  SV_TRY(msm_batch_fixed_device(t.pre, t.n, sg.at<const uint32_t>(0), sg.at(1), sg.at<const uint64_t>(2), count, form,
                                t.dev, nullptr, sg.at(3)));
  SV_TRY(sg.get(out, 3, count * sizeof(sv_g1_affine)));
  SV_TRY(sg.sync());
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_batch_table_device(uint64_t handle, const uint32_t* d_base_idx, const sv_fe* d_scalars,
                                       const uint64_t* d_offsets, size_t count, int form, void* stream,
                                       sv_g1_affine* d_out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (count == 0) return SV_OK;
  if (!d_base_idx || !d_scalars || !d_offsets || !d_out) return SV_ERR_ARG;
  BaseTable t;
  if (!table_lookup(handle, &t)) {
    sv::set_error("unknown base table handle %llu", (unsigned long long)handle);
    return SV_ERR_ARG;
  }
  SV_HIP(hipSetDevice(t.dev));
  return msm_batch_fixed_device(t.pre, t.n, d_base_idx, d_scalars, d_offsets, count, form, t.dev,
                                (hipStream_t)stream, d_out);
  SV_GUARD_END
}

int sv_bn254_g1_table_device(uint64_t handle, int* device) noexcept {
  SV_GUARD_BEGIN
  BaseTable t;
  if (!device || !table_lookup(handle, &t)) {
    sv::set_error("unknown base table handle %llu", (unsigned long long)handle);
    return SV_ERR_ARG;
  }
  *device = t.dev;
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_msm_batch_indexed_device(const sv_g1_affine* d_table, size_t table_len, int table_form,
                                         const uint32_t* d_base_idx, const sv_fe* d_scalars,
                                         const uint64_t* d_offsets, size_t count, size_t max_terms, int form,
                                         int device, void* stream, sv_g1_affine* d_out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  SV_TRY(check_form(table_form));
  if (count == 0) return SV_OK;
  if (!d_table || !d_base_idx || !d_scalars || !d_offsets || !d_out) return SV_ERR_ARG;
  if (table_len == 0) {
    sv::set_error("empty base table");
    return SV_ERR_EMPTY;
  }
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  SV_HIP(hipSetDevice(device));
  return msm_batch_device(d_table, d_scalars, d_offsets, nullptr, count, max_terms, form, device,
                          (hipStream_t)stream, d_out, d_base_idx, table_len, table_form);
  SV_GUARD_END
}

int sv_bn254_poseidon_permute(sv_fe* states, size_t n, int t, int form) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (t != 3 && t != 5) {
    sv::set_error("poseidon: unsupported width t = %d (3 or 5)", t);
    return SV_ERR_ARG;
  }
  if (n == 0) return SV_OK;
  if (!states) return SV_ERR_ARG;
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  const size_t bytes = n * (size_t)t * sizeof(sv_fe);
  Staging sg(dev);
  SV_TRY(sg.init({bytes}));
  SV_TRY(sg.put(0, states, bytes));
  SV_TRY(poseidon_permute_device(sg.at(0), n, t, form, sg.lease.get()->stream));
  SV_TRY(sg.get(states, 0, bytes));
  SV_TRY(sg.sync());
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_poseidon_permute_device(sv_fe* d_states, size_t n, int t, int form, int device, void* stream) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  SV_HIP(hipSetDevice(device));
  return poseidon_permute_device(d_states, n, t, form, (hipStream_t)stream);
  SV_GUARD_END
}

int sv_bn254_poseidon_squeeze(sv_fe* states, const sv_fe* elements, const uint64_t* offsets, size_t n, int t,
                              int form, sv_fe* out) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (t != 3 && t != 5) {
    sv::set_error("poseidon: unsupported width t = %d (3 or 5)", t);
    return SV_ERR_ARG;
  }
  if (n == 0) return SV_OK;
  if (!states || !offsets) return SV_ERR_ARG;
  for (size_t j = 0; j < n; j++)
    if (offsets[j + 1] < offsets[j]) {
      sv::set_error("poseidon: offsets not non-decreasing at %zu", j);
      return SV_ERR_ARG;
    }
  const uint64_t total = offsets[n] - offsets[0];
  if (total && !elements) return SV_ERR_ARG;
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  // rebase offsets so only elements[offsets[0] .. offsets[n]) travel
  std::vector<uint64_t> off(offsets, offsets + n + 1);
  for (auto& o : off) o -= offsets[0];
  const size_t sbytes = n * (size_t)t * sizeof(sv_fe);
  Staging sg(dev);
  SV_TRY(sg.init({sbytes, total * sizeof(sv_fe), (n + 1) * sizeof(uint64_t), n * sizeof(sv_fe)}));
  SV_TRY(sg.put(0, states, sbytes));
  if (total) SV_TRY(sg.put(1, elements + offsets[0], total * sizeof(sv_fe)));
  SV_TRY(sg.put(2, off.data(), (n + 1) * sizeof(uint64_t)));
  SV_TRY(poseidon_squeeze_device(sg.at(0), sg.at(1), sg.at<const uint64_t>(2), n, t, form, sg.at(3),
                                 sg.lease.get()->stream));
  SV_TRY(sg.get(states, 0, sbytes));
  if (out) SV_TRY(sg.get(out, 3, n * sizeof(sv_fe)));
  SV_TRY(sg.sync());
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_poseidon_squeeze_device(sv_fe* d_states, const sv_fe* d_elements, const uint64_t* d_offsets, size_t n,
                                     int t, int form, sv_fe* d_out, int device, void* stream) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  SV_HIP(hipSetDevice(device));
  return poseidon_squeeze_device(d_states, d_elements, d_offsets, n, t, form, d_out, (hipStream_t)stream);
  SV_GUARD_END
}

int sv_bn254_g1_decode(const uint8_t* data, size_t n, int encoding, int form, sv_g1_affine* out,
                       int64_t* first_invalid) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (encoding != SV_ENC_HALO2_COMPRESSED && encoding != SV_ENC_EVM) {
    sv::set_error("unknown point encoding %d", encoding);
    return SV_ERR_ARG;
  }
  int64_t fi = -1;
  if (first_invalid) *first_invalid = -1;
  if (n == 0) return SV_OK;
  if (!data || !out) return SV_ERR_ARG;
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  const size_t rec = encoding == SV_ENC_EVM ? 64 : 32;
  Staging sg(dev);
  SV_TRY(sg.init({n * rec, n * sizeof(sv_g1_affine)}));
  SV_TRY(sg.put(0, data, n * rec));
  SV_TRY(sg.sync());
  SV_TRY(g1_decode_device(sg.at(0), n, encoding, rec, 0, form, dev, nullptr, sg.at(1), &fi));
  SV_TRY(sg.get(out, 1, n * sizeof(sv_g1_affine)));
  SV_TRY(sg.sync());
  if (first_invalid) *first_invalid = fi;
  if (fi >= 0) {
    sv::set_error("Invalid elliptic curve point encoding in proof (point %lld)", (long long)fi);
    return SV_ERR_ARG;
  }
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_g1_decode_device(const uint8_t* d_data, size_t n, int encoding, int form, int device, void* stream,
                              sv_g1_affine* d_out, int64_t* first_invalid) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  SV_HIP(hipSetDevice(device));
  int64_t fi = -1;
  SV_TRY(g1_decode_device(d_data, n, encoding, encoding == SV_ENC_EVM ? 64 : 32, 0, form, device,
                          (hipStream_t)stream, d_out, &fi));
  if (first_invalid) *first_invalid = fi;
  if (fi >= 0) {
    sv::set_error("Invalid elliptic curve point encoding in proof (point %lld)", (long long)fi);
    return SV_ERR_ARG;
  }
  return SV_OK;
  SV_GUARD_END
}

int sv_bn254_kzg_accumulators_from_limbs(const sv_fe* limbs, size_t n, int n_limbs, int bits, int form,
                                         sv_g1_affine* lhs, sv_g1_affine* rhs, int64_t* first_invalid) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (first_invalid) *first_invalid = -1;
  if (n == 0) return SV_OK;
  if (!limbs || !lhs || !rhs || n_limbs < 1) return SV_ERR_ARG;
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  const size_t nl = n * 4 * (size_t)n_limbs;
  Staging sg(dev);
  SV_TRY(sg.init({nl * sizeof(sv_fe), n * sizeof(sv_g1_affine), n * sizeof(sv_g1_affine)}));
  SV_TRY(sg.put(0, limbs, nl * sizeof(sv_fe)));
  SV_TRY(sg.sync());
  int64_t fi = -1;
  SV_TRY(limbs_to_accumulators_device(sg.at(0), n, n_limbs, bits, form, dev, nullptr, sg.at(1), sg.at(2), &fi));
  SV_TRY(sg.get(lhs, 1, n * sizeof(sv_g1_affine)));
  SV_TRY(sg.get(rhs, 2, n * sizeof(sv_g1_affine)));
  SV_TRY(sg.sync());
  if (first_invalid) *first_invalid = fi;
  if (fi >= 0) {
    sv::set_error("accumulator %lld: limbs do not encode a canonical on-curve point", (long long)fi);
    return SV_ERR_ARG;
  }
  return SV_OK;
  SV_GUARD_END
}

namespace {
// 32-byte big-endian word -> canonical limbs; false when >= p
bool be_word(const uint8_t* w, F& out) {
  for (int k = 0; k < 4; k++) {
    uint64_t v = 0;
    for (int b = 0; b < 8; b++) v = (v << 8) | w[(3 - k) * 8 + b];
    out.l[k] = v;
  }
  return host::f_is_reduced(out);
}
bool g2_from_eip197(const uint8_t* r, sv_g2_affine* q) {
  F w[4];
  for (int i = 0; i < 4; i++)
    if (!be_word(r + 32 * i, w[i])) return false;
  q->x.c1 = fe_out(w[0]);
  q->x.c0 = fe_out(w[1]);
  q->y.c1 = fe_out(w[2]);
  q->y.c0 = fe_out(w[3]);
  return true;
}
}  // namespace

int sv_bn254_kzg_decide_eip197(const uint8_t* input, size_t n_checks, int num_gpus, int32_t* first_fail) noexcept {
  SV_GUARD_BEGIN
  (void)num_gpus;  // one device: the records are host memory and the check count is small
  if (n_checks == 0) {
    sv::set_error("accumulators should not be empty");
    return SV_ERR_EMPTY;
  }
  if (!input || !first_fail) return SV_ERR_ARG;
  constexpr size_t kRec = 0x180;
  sv_g2_affine g2, msg2;
  if (!g2_from_eip197(input + 64, &g2) || !g2_from_eip197(input + 256, &msg2)) {
    sv::set_error("EIP-197 record 0: G2 word >= p");
    return SV_ERR_ARG;
  }
  for (size_t i = 1; i < n_checks; i++)
    if (memcmp(input + i * kRec + 64, input + 64, 128) || memcmp(input + i * kRec + 256, input + 256, 128)) {
      sv::set_error("EIP-197 record %zu: G2 points differ from record 0 (one deciding key per call)", i);
      return SV_ERR_ARG;
    }
  // s_g2 = -(-s_g2): negate y (canonical)
  sv_g2_affine sg2 = msg2;
  {
    F y0 = fe_in(msg2.y.c0), y1 = fe_in(msg2.y.c1);
    sg2.y.c0 = fe_out(host::f_sub(F{}, y0));
    sg2.y.c1 = fe_out(host::f_sub(F{}, y1));
  }
  if (resolve_gpus(1) == 0) return SV_ERR_DEVICE;
  const int dev = runtime_device_id(0);
  Staging sg(dev);
  SV_TRY(sg.init({n_checks * kRec, n_checks * sizeof(sv_g1_affine), n_checks * sizeof(sv_g1_affine)}));
  SV_TRY(sg.put(0, input, n_checks * kRec));
  SV_TRY(sg.sync());
  int64_t bl = -1, br = -1;
  SV_TRY(g1_decode_device(sg.at(0), n_checks, SV_ENC_EVM, kRec, 0, SV_CANONICAL, dev, nullptr, sg.at(1), &bl));
  SV_TRY(g1_decode_device(sg.at(0), n_checks, SV_ENC_EVM, kRec, 192, SV_CANONICAL, dev, nullptr, sg.at(2), &br));
  int32_t ff = -1;
  SV_TRY(decide_run_device(&g2, &sg2, sg.at(1), sg.at(2), n_checks, SV_CANONICAL, dev, nullptr, &ff, nullptr,
                           nullptr));
  int64_t first = -1;
  for (int64_t c : {(int64_t)ff, bl, br})
    if (c >= 0 && (first < 0 || c < first)) first = c;
  *first_fail = (int32_t)first;
  return SV_OK;
  SV_GUARD_END
}

int sv_gen_scalars_device(sv_fe* d_scalars, size_t n, uint64_t seed, uint64_t start, int form, int device,
                          void* stream) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  return gen_scalars_device(d_scalars, n, seed, start, form, device, (hipStream_t)stream);
  SV_GUARD_END
}

int sv_gen_bases_device(sv_g1_affine* d_bases, size_t n, uint64_t seed, uint64_t start, int form, int device,
                        void* stream) noexcept {
  SV_GUARD_BEGIN
  SV_TRY(check_form(form));
  if (resolve_gpus(0) == 0) return SV_ERR_DEVICE;
  return gen_bases_device(d_bases, n, seed, start, form, device, (hipStream_t)stream);
  SV_GUARD_END
}

int sv_msm_last_stats(sv_msm_stats* out) noexcept {
  SV_GUARD_BEGIN
  if (!out) return SV_ERR_ARG;
  return msm_last_stats(out);
  SV_GUARD_END
}

int sv_kzg_last_kernel_ms(float* out) noexcept {
  if (!out) return SV_ERR_ARG;
  *out = decider_last_kernel_ms();
  return SV_OK;
}

}  // extern "C"
