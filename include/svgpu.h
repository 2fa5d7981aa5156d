/*
 * svgpu.h -- C ABI of the MI355X-native BN254 MSM + KZG-decider backend (libsvgpu.so).
 *
 * Drop-in boundary for snark-verifier's native hot path (yuliakot/snark-verifier-axiom):
 *
 *   sv_bn254_g1_msm          replaces  NativeLoader::multi_scalar_multiplication
 *                                      snark-verifier/src/loader/native.rs:61-71
 *                            and       util::msm::multi_scalar_multiplication
 *                                      snark-verifier/src/util/msm.rs:287-316
 *   sv_bn254_kzg_decide      replaces  AccumulationDecider::{decide, decide_all} for KzgAs on NativeLoader
 *                                      snark-verifier/src/pcs/kzg/decider.rs:60-68 and :70-80
 *   sv_bn254_kzg_accumulate  replaces  KzgAs::create_proof's two MSMs (no zk blind)
 *   sv_bn254_kzg_create_proof   the same with r squeezed from the Poseidon transcript
 *                                      snark-verifier/src/pcs/kzg/accumulation.rs:146-195
 *                                      (also AccumulationScheme::verify, :40-62)
 *
 * The Rust binding a maintainer adds is in INTEGRATION.md.  Conventions:
 *  - every function is extern "C", never throws, and returns an sv_status;
 *  - every pointer is caller-owned and borrowed for the call only; nothing is retained;
 *  - field elements are 4 x u64 little-endian limbs (= halo2curves' in-memory Fq/Fr layout);
 *    `form` says whether inputs/outputs are canonical (SV_CANONICAL) or Montgomery with
 *    R = 2^256 (SV_MONTGOMERY, zero-copy with halo2curves memory);
 *  - the affine identity is (0, 0), as halo2curves encodes it;
 *  - calls are re-entrant: each call draws a stream + workspace from a per-device pool.
 *  - there is NO CPU fallback inside this library: without a usable GPU every compute entry
 *    point returns SV_ERR_DEVICE (the Rust shim then keeps the reference's own CPU code path).
 */
#ifndef SVGPU_H_
#define SVGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define SV_NOEXCEPT noexcept
extern "C" {
#else
#define SV_NOEXCEPT
#endif

#define SVGPU_ABI_VERSION 1

typedef struct { uint64_t l[4]; } sv_fe;                 /* Fq or Fr element                     */
typedef struct { sv_fe x, y; } sv_g1_affine;             /* identity = all-zero                  */
typedef struct { sv_fe x, y, z; } sv_g1_jacobian;        /* x = X/Z^2, y = Y/Z^3; identity Z = 0 */
typedef struct { sv_fe c0, c1; } sv_fq2;                 /* c0 + c1*u, u^2 = -1                  */
typedef struct { sv_fq2 x, y; } sv_g2_affine;            /* D-type twist coords; identity = 0    */
typedef struct { sv_fq2 c[6]; } sv_fq12;                 /* c0.c0 c0.c1 c0.c2 c1.c0 c1.c1 c1.c2  */

enum sv_form { SV_CANONICAL = 0, SV_MONTGOMERY = 1 };

enum sv_status {
  SV_OK = 0,
  SV_ERR_EMPTY = 1,  /* n == 0: "pairs should not be empty" (native.rs:69) / decider.rs:74 */
  SV_ERR_LEN = 2,    /* size too large for the device workspace                            */
  SV_ERR_ARG = 3,    /* null pointer, bad form, non-reduced element, point not on curve    */
  SV_ERR_DEVICE = 4, /* no usable GPU, or a HIP runtime error                              */
  SV_ERR_OOM = 5     /* device allocation failed                                           */
};

/* ---- runtime ---------------------------------------------------------------------- */
int sv_init(int num_devices) SV_NOEXCEPT;        /* idempotent; <= 0 means every visible device      */
int sv_device_count(void) SV_NOEXCEPT;           /* devices initialised (0 before sv_init / no GPU)  */
const char* sv_last_error(void) SV_NOEXCEPT;     /* thread-local message for the last non-OK status  */
const char* sv_version(void) SV_NOEXCEPT;

/* ---- a1/a3: multi-scalar multiplication ---------------------------------------------
 * out = sum_i scalars[i] * bases[i] as an affine point (identity -> (0,0)).
 * Host buffers.  num_gpus <= 0 means every initialised device (point-sharded, partials
 * folded in device order).  Scalars must be reduced (< r) and base coordinates reduced
 * (< p) in the given form, else SV_ERR_ARG.  The inputs reach HBM in pieces on a copy
 * stream (default: 4 pieces weighted 5,4,4,3 from 2^18 points, 2 equal from 2^15, else 1;
 * SVGPU_H2D_PIECES = N equal pieces, SVGPU_H2D_SPLIT = comma-separated weights); each
 * piece is sorted on a second stream once its scalars land and accumulated into the one
 * bucket set once its bases land, while later pieces are in flight; buffers are pooled.   */
int sv_bn254_g1_msm(const sv_g1_affine* bases, const sv_fe* scalars, size_t n, int form,
                    int num_gpus, sv_g1_affine* out) SV_NOEXCEPT;

/* The same MSM over the exact shape NativeLoader::multi_scalar_multiplication receives
 * (native.rs:61-71: pairs: &[(&Fr, &G1Affine)], an array of references into scattered
 * caller memory).  The library gathers the referenced 96 B per pair on its host worker pool
 * straight into pinned staging, piece by piece, and each piece's DMA and sort overlap the
 * gather of the next -- the shim passes its pairs as this 16-B-per-pair struct array (a Rust
 * tuple's field order is unspecified, so the shim maps (&Fr, &G1Affine) into sv_msm_ref).
 * A NULL reference is SV_ERR_ARG.                                                          */
typedef struct { const sv_fe* scalar; const sv_g1_affine* base; } sv_msm_ref;
int sv_bn254_g1_msm_refs(const sv_msm_ref* pairs, size_t n, int form, int num_gpus,
                         sv_g1_affine* out) SV_NOEXCEPT;

/* Device-resident variant (bases/scalars already in HBM on `device`, `stream` may be NULL):
 * writes this shard's partial sum to *out_partial (host memory, Jacobian, canonical form).
 * This is the per-rank step of the RCCL-sharded MSM (one process per GPU).              */
int sv_bn254_g1_msm_device(const sv_g1_affine* d_bases, const sv_fe* d_scalars, size_t n,
                           int form, int device, void* stream, sv_g1_jacobian* out_partial) SV_NOEXCEPT;

/* Fold Jacobian partials (canonical form) in index order and convert to affine.  Host-only
 * (no GPU needed): the combine step after the RCCL all-gather of per-rank partials.      */
int sv_bn254_g1_fold(const sv_g1_jacobian* partials, size_t k, sv_g1_affine* out, int out_form) SV_NOEXCEPT;

/* ---- a7/a8: KZG decider ----------------------------------------------------------------
 * For every i: e(lhs[i], g2) * e(rhs[i], -s_g2) == 1 ?  *first_fail = first failing index, or
 * -1 when all pass (the reference returns Err(AssertionFailure) on the first failure).
 * Identity G1 inputs contribute 1, as halo2curves' multi_miller_loop skips them.          */
int sv_bn254_kzg_decide(const sv_g2_affine* g2, const sv_g2_affine* s_g2,
                        const sv_g1_affine* lhs, const sv_g1_affine* rhs, size_t n, int form,
                        int num_gpus, int32_t* first_fail) SV_NOEXCEPT;

/* Device-resident variant; optional per-accumulator outputs:
 *   verdicts (host, n int32: 1 = pass) and gt (host, n sv_fq12, canonical: the value
 *   e(lhs,g2)*e(rhs,-s_g2) after final exponentiation, for Gt-value parity tests).        */
int sv_bn254_kzg_decide_device(const sv_g2_affine* g2, const sv_g2_affine* s_g2,
                               const sv_g1_affine* d_lhs, const sv_g1_affine* d_rhs, size_t n,
                               int form, int device, void* stream, int32_t* first_fail,
                               int32_t* verdicts, sv_fq12* gt) SV_NOEXCEPT;

/* ---- a10: KZG accumulation (KzgAs::create_proof / verify without blind) -----------------
 * out_lhs = sum_i r^i lhs[i], out_rhs = sum_i r^i rhs[i], r^0 = 1 (loader.rs:71-78).       */
int sv_bn254_kzg_accumulate(const sv_g1_affine* lhs, const sv_g1_affine* rhs, size_t n,
                            const sv_fe* r, int form, int num_gpus, sv_g1_affine* out_lhs,
                            sv_g1_affine* out_rhs) SV_NOEXCEPT;

/* KzgAs::create_proof without blind, challenge included (accumulation.rs:146-195): a fresh
 * Poseidon transcript (T = 3, RATE = 2, R_F = 8, R_P = 57, snark-verifier-sdk/src/halo2.rs:52-55)
 * absorbs lhs[i], rhs[i] for i = 0..n through common_ec_point (x, y as Fq -> Fr mod r,
 * system/halo2/transcript/halo2.rs:214-226), squeezes r (accumulation.rs:176), then returns the
 * sv_bn254_kzg_accumulate result for that r.  sponge_state (3 elements in `form`, may be
 * NULL = a fresh transcript, Poseidon::new's (2^64, 0, 0)) is the transcript's sponge state before
 * the call and receives it after the squeeze, for a transcript that was squeezed before (its
 * buffer empty).  out_r (may be NULL) receives r in `form`.  An identity accumulator point is
 * SV_ERR_ARG (the reference's Error::Transcript, halo2.rs:215-223).  The sponge (n + 1 dependent
 * permutations) runs on the host; the MSMs on the device.                                    */
int sv_bn254_kzg_create_proof(const sv_g1_affine* lhs, const sv_g1_affine* rhs, size_t n, int form,
                              int num_gpus, sv_g1_affine* out_lhs, sv_g1_affine* out_rhs,
                              sv_fe* sponge_state, sv_fe* out_r) SV_NOEXCEPT;

/* ---- batched small MSMs -------------------------------------
 * count independent MSMs over shared arrays: MSM k = sum_{i in [offsets[k], offsets[k+1])}
 * scalars[i] * bases[i]; offsets has count + 1 non-decreasing entries; out[k] affine in
 * `form`.  The per-proof Msm::evaluate calls of a native verifier (bdfg21.rs:75-78,
 * gwc19.rs:76-79 -> native.rs:61-71) and the two accumulation MSMs of KzgAs::create_proof
 * (accumulation.rs:177-192) in one launch.  An empty MSM is SV_ERR_EMPTY ("pairs should not
 * be empty", native.rs:69).  Host API: MSMs above SVGPU_BATCH_MAX terms (default 4096), and
 * every MSM of a batch of at most SVGPU_BATCH_SEQ_MAX (default 4), run through the single-MSM
 * pipeline instead.  Device API: every MSM runs in the batch kernel
 * (max_terms = the largest MSM, picks the window size); synchronous on `stream`.          */
int sv_bn254_g1_msm_batch(const sv_g1_affine* bases, const sv_fe* scalars, const uint64_t* offsets,
                          size_t count, int form, sv_g1_affine* out) SV_NOEXCEPT;
int sv_bn254_g1_msm_batch_device(const sv_g1_affine* d_bases, const sv_fe* d_scalars,
                                 const uint64_t* d_offsets, size_t count, size_t max_terms,
                                 int form, int device, void* stream,
                                 sv_g1_affine* d_out) SV_NOEXCEPT;

/* ---- device-resident fixed bases for batched MSMs ------------
 * A native verifier's constant bases -- the generator and the circuit's preprocessed
 * commitments, loaded once per verifier (Protocol::loaded, plonk/protocol.rs:106-131; used by
 * the per-proof Msm::evaluate of bdfg21.rs:75-78 / gwc19.rs:76-79) -- are uploaded ONCE as a
 * base table (stored in Montgomery form on `device`; coordinates must be reduced) and then
 * referenced by index, so a per-proof batch ships only scalars and u32 indices:
 *   MSM k = sum_{i in [offsets[k], offsets[k+1])} scalars[i] * table[base_idx[i]].
 * An index >= the table length is SV_ERR_ARG; an empty MSM is SV_ERR_EMPTY.  Handles are
 * process-wide and thread-safe; a destroyed or unknown handle is SV_ERR_ARG.              */
int sv_bn254_g1_table_create(const sv_g1_affine* bases, size_t n, int form, int device,
                             uint64_t* handle) SV_NOEXCEPT;
int sv_bn254_g1_table_destroy(uint64_t handle) SV_NOEXCEPT;
int sv_bn254_g1_msm_batch_table(uint64_t handle, const uint32_t* base_idx, const sv_fe* scalars,
                                const uint64_t* offsets, size_t count, int form,
                                sv_g1_affine* out) SV_NOEXCEPT;
/* Table rows are precomputed at creation as their window multiples 2^(8 w) P (w < 32, affine,
 * 2 KiB per row on the device), so a table-backed MSM puts every signed 8-bit digit of every
 * term into ONE bucket set (no per-MSM Horner over windows).  Device-buffer form of the same:
 * d_base_idx / d_scalars / d_offsets (count + 1 entries) / d_out on the table's device
 * (sv_bn254_g1_table_device), synchronous on `stream`; an empty MSM gives the identity.     */
int sv_bn254_g1_msm_batch_table_device(uint64_t handle, const uint32_t* d_base_idx, const sv_fe* d_scalars,
                                       const uint64_t* d_offsets, size_t count, int form, void* stream,
                                       sv_g1_affine* d_out) SV_NOEXCEPT;
int sv_bn254_g1_table_device(uint64_t handle, int* device) SV_NOEXCEPT;
/* device-buffer form over a raw (not precomputed) table: d_table (table_len rows, `table_form`), d_base_idx / d_scalars / d_offsets /
 * d_out on `device`; max_terms = the largest MSM (picks the window size); synchronous.        */
int sv_bn254_g1_msm_batch_indexed_device(const sv_g1_affine* d_table, size_t table_len, int table_form,
                                         const uint32_t* d_base_idx, const sv_fe* d_scalars,
                                         const uint64_t* d_offsets, size_t count, size_t max_terms,
                                         int form, int device, void* stream,
                                         sv_g1_affine* d_out) SV_NOEXCEPT;

/* ---- Poseidon sponge over BN254 Fr --------------------------
 * x^5 HADES permutation, width t = 3 (R_F 8, R_P 57, rate 2: the SDK's PoseidonTranscript,
 * snark-verifier-sdk/src/halo2.rs:52-71) or t = 5 (R_F 8, R_P 60, rate 4).  States are t
 * consecutive sv_fe; inputs must be reduced field elements.
 * permute: the bare HADES permutation of n states, in place: Poseidon::permutation
 *          (snark-verifier/src/util/hash/poseidon.rs:469-500) called with a full-rate zero
 *          input, exactly as the reference KATs call it (poseidon/tests.rs:34-85).
 * squeeze: Poseidon::squeeze (poseidon.rs:455-467) on n independent sponges.  states (n x t,
 *          in/out) are the sponges' states -- Poseidon::new starts one at (2^64, 0, ..),
 *          poseidon.rs:335-342 -- and sponge j's buffer (what Poseidon::update collected,
 *          poseidon.rs:449-452) is elements[offsets[j] .. offsets[j+1]); offsets has n + 1
 *          non-decreasing entries.  out[j] (optional, may be NULL) = the challenge state[1].  */
int sv_bn254_poseidon_permute(sv_fe* states, size_t n, int t, int form) SV_NOEXCEPT;
int sv_bn254_poseidon_permute_device(sv_fe* d_states, size_t n, int t, int form, int device,
                                     void* stream) SV_NOEXCEPT;
int sv_bn254_poseidon_squeeze(sv_fe* states, const sv_fe* elements, const uint64_t* offsets,
                              size_t n, int t, int form, sv_fe* out) SV_NOEXCEPT;
int sv_bn254_poseidon_squeeze_device(sv_fe* d_states, const sv_fe* d_elements,
                                     const uint64_t* d_offsets, size_t n, int t, int form,
                                     sv_fe* d_out, int device, void* stream) SV_NOEXCEPT;

/* ---- codecs around the path, decoded on the device --------
 * Point encodings:
 *   SV_ENC_HALO2_COMPRESSED  32 B: x little-endian, parity of y in bit 255, identity = zeros
 *                            (halo2curves GroupEncoding, read by PoseidonTranscript::read_ec_point,
 *                            system/halo2/transcript/halo2.rs:247-260)
 *   SV_ENC_EVM               64 B: x || y big-endian, identity = zeros
 *                            (EvmTranscript::read_ec_point, system/halo2/transcript/evm.rs:223-242)
 * g1_decode: n encoded points -> affine in `form`.  All valid: SV_OK and *first_invalid = -1.
 *   Otherwise SV_ERR_ARG ("Invalid elliptic curve point encoding in proof"), *first_invalid =
 *   the lowest invalid index, and invalid points are written as (0, 0).
 * accumulators_from_limbs: LimbsEncoding<LIMBS, BITS>::from_repr (pcs/kzg/accumulator.rs:57-77)
 *   for n accumulators of 4 * n_limbs Fr limbs each (lhs.x, lhs.y, rhs.x, rhs.y; fe_from_limbs,
 *   util/arithmetic.rs:262-274; the SDK uses LIMBS = 3, BITS = 88).  `form` applies to the limbs
 *   and the output.  A coordinate >= p or >= 2^256, or a point off the curve (the reference's
 *   unwrap panics) gives SV_ERR_ARG with *first_invalid = that accumulator.
 * kzg_decide_eip197: n_checks 0x180-byte ecPairing (EIP-197) inputs as the EVM decider lays them
 *   out (pcs/kzg/decider.rs:107-127, loader/evm/loader.rs:338-382): lhs, g2, rhs, -s_g2 with G2
 *   words (x.c1, x.c0, y.c1, y.c0).  All records must carry the same G2 pair (one deciding key).
 *   *first_fail = first check whose pairing product is not 1 or whose G1 encoding is invalid
 *   (the precompile would fail either way), -1 if all pass.                             */
enum { SV_ENC_HALO2_COMPRESSED = 0, SV_ENC_EVM = 1 };
int sv_bn254_g1_decode(const uint8_t* data, size_t n, int encoding, int form, sv_g1_affine* out,
                       int64_t* first_invalid) SV_NOEXCEPT;
int sv_bn254_g1_decode_device(const uint8_t* d_data, size_t n, int encoding, int form, int device,
                              void* stream, sv_g1_affine* d_out,
                              int64_t* first_invalid) SV_NOEXCEPT;
int sv_bn254_kzg_accumulators_from_limbs(const sv_fe* limbs, size_t n, int n_limbs, int bits,
                                         int form, sv_g1_affine* lhs, sv_g1_affine* rhs,
                                         int64_t* first_invalid) SV_NOEXCEPT;
int sv_bn254_kzg_decide_eip197(const uint8_t* input, size_t n_checks, int num_gpus,
                               int32_t* first_fail) SV_NOEXCEPT;

/* ---- synthetic inputs (SURVEY.md section 8d generator, index-addressable) -------------
 * Fills device buffers with the deterministic SplitMix64 scalars / try-and-increment bases
 * (elements start .. start+n-1) in the requested form.                                   */
int sv_gen_scalars_device(sv_fe* d_scalars, size_t n, uint64_t seed, uint64_t start, int form,
                          int device, void* stream) SV_NOEXCEPT;
int sv_gen_bases_device(sv_g1_affine* d_bases, size_t n, uint64_t seed, uint64_t start, int form,
                        int device, void* stream) SV_NOEXCEPT;

/* ---- instrumentation ----------------------------------------------------------------
 * Per-kernel timings (HIP events on the call's stream) of the last MSM on this thread; the digits
 * and fixup splits are filled only with SVGPU_MSM_STATS=1 (folded into sort / reduce otherwise). */
typedef struct {
  float total_ms, digits_ms, sort_ms, accumulate_ms, fixup_ms, reduce_ms, host_ms;
  uint32_t window_bits, num_windows, accumulate_launch_units;
  uint64_t entries;
  float accumulate_span_ms;        /* first accumulate launch's start to the last one's end */
  uint32_t accumulate_launches;    /* 2 when the window halves run as separate launches */
} sv_msm_stats;
int sv_msm_last_stats(sv_msm_stats* out) SV_NOEXCEPT;
/* Kernel time (HIP events on the call's stream) of the calling thread's last decider launch. */
int sv_kzg_last_kernel_ms(float* out) SV_NOEXCEPT;

#ifdef __cplusplus
}
#endif
#endif /* SVGPU_H_ */
