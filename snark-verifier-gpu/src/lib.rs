//! `snark-verifier-gpu`: the FFI crate over libsvgpu.so (include/svgpu.h) that snark-verifier's
//! `gpu` feature calls.  snark-verifier itself forbids unsafe code (snark-verifier/src/lib.rs:3),
//! so every `unsafe` block of the integration lives here.  See INTEGRATION.md for the three call
//! sites (loader/native.rs:61-71, util/msm.rs:287, pcs/kzg/decider.rs:60-80).
//!
//! Not compiled in this repository's image (no Rust toolchain); tests/test_rust_shim.py checks
//! that this file declares every C-ABI function of include/svgpu.h with the same arity, and the
//! parity of every entry point is proven at the C ABI by tests/ (through the same libsvgpu.so).
//!
//! Every safe wrapper returns `None` on a device error (no GPU, HIP error) so the caller keeps
//! the reference's own CPU path; reference panics (empty input) are reproduced as panics.
//!
//! Toolchain: the crate builds with the reference's pinned `nightly-2022-10-28`
//! (`rust-toolchain`), so it uses only std items stable at that date and enables no nightly
//! feature: process-wide lazy values are `std::sync::Once` + atomics, not `OnceLock` (stable
//! only from 1.70).  tests/test_rust_shim.py keeps a denylist of later std items.
#![allow(clippy::missing_safety_doc)]

use halo2curves::bn256::{Fq, Fr, G1Affine, G2Affine};
use halo2curves::pairing::Engine;
use halo2curves::CurveAffine;
use std::os::raw::{c_char, c_int, c_void};
use std::sync::atomic::{AtomicBool, AtomicUsize, Ordering};
use std::sync::Once;

pub const SV_CANONICAL: c_int = 0;
pub const SV_MONTGOMERY: c_int = 1;
pub const SV_OK: c_int = 0;
pub const SV_ERR_EMPTY: c_int = 1;
pub const SV_ERR_LEN: c_int = 2;
pub const SV_ERR_ARG: c_int = 3;
pub const SV_ERR_DEVICE: c_int = 4;
pub const SV_ERR_OOM: c_int = 5;
pub const SV_ENC_HALO2_COMPRESSED: c_int = 0;
pub const SV_ENC_EVM: c_int = 1;

#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct SvFe {
    pub l: [u64; 4],
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug, PartialEq, Eq)]
pub struct SvG1Affine {
    pub x: SvFe,
    pub y: SvFe,
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct SvG1Jacobian {
    pub x: SvFe,
    pub y: SvFe,
    pub z: SvFe,
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct SvFq2 {
    pub c0: SvFe,
    pub c1: SvFe,
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct SvG2Affine {
    pub x: SvFq2,
    pub y: SvFq2,
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct SvFq12 {
    pub c: [SvFq2; 6],
}
/// One (&Fr, &G1Affine) pair of NativeLoader::multi_scalar_multiplication (native.rs:61-71).
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct SvMsmRef {
    pub scalar: *const SvFe,
    pub base: *const SvG1Affine,
}
#[repr(C)]
#[derive(Clone, Copy, Default, Debug)]
pub struct SvMsmStats {
    pub total_ms: f32,
    pub digits_ms: f32,
    pub sort_ms: f32,
    pub accumulate_ms: f32,
    pub fixup_ms: f32,
    pub reduce_ms: f32,
    pub host_ms: f32,
    pub window_bits: u32,
    pub num_windows: u32,
    pub accumulate_launch_units: u32,
    pub entries: u64,
    pub accumulate_span_ms: f32,
    pub accumulate_launches: u32,
}

#[link(name = "svgpu")]
extern "C" {
    pub fn sv_init(num_devices: c_int) -> c_int;
    pub fn sv_device_count() -> c_int;
    pub fn sv_last_error() -> *const c_char;
    pub fn sv_version() -> *const c_char;
    pub fn sv_bn254_g1_msm(bases: *const SvG1Affine, scalars: *const SvFe, n: usize, form: c_int,
                           num_gpus: c_int, out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_msm_refs(pairs: *const SvMsmRef, n: usize, form: c_int, num_gpus: c_int,
                                out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_msm_device(d_bases: *const SvG1Affine, d_scalars: *const SvFe, n: usize, form: c_int,
                                  device: c_int, stream: *mut c_void, out_partial: *mut SvG1Jacobian) -> c_int;
    pub fn sv_bn254_g1_fold(partials: *const SvG1Jacobian, k: usize, out: *mut SvG1Affine, out_form: c_int) -> c_int;
    pub fn sv_bn254_kzg_decide(g2: *const SvG2Affine, s_g2: *const SvG2Affine, lhs: *const SvG1Affine,
                               rhs: *const SvG1Affine, n: usize, form: c_int, num_gpus: c_int,
                               first_fail: *mut i32) -> c_int;
    pub fn sv_bn254_kzg_decide_device(g2: *const SvG2Affine, s_g2: *const SvG2Affine, d_lhs: *const SvG1Affine,
                                      d_rhs: *const SvG1Affine, n: usize, form: c_int, device: c_int,
                                      stream: *mut c_void, first_fail: *mut i32, verdicts: *mut i32,
                                      gt: *mut SvFq12) -> c_int;
    pub fn sv_bn254_kzg_accumulate(lhs: *const SvG1Affine, rhs: *const SvG1Affine, n: usize, r: *const SvFe,
                                   form: c_int, num_gpus: c_int, out_lhs: *mut SvG1Affine,
                                   out_rhs: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_kzg_create_proof(lhs: *const SvG1Affine, rhs: *const SvG1Affine, n: usize, form: c_int,
                                     num_gpus: c_int, out_lhs: *mut SvG1Affine, out_rhs: *mut SvG1Affine,
                                     sponge_state: *mut SvFe, out_r: *mut SvFe) -> c_int;
    pub fn sv_bn254_g1_msm_batch(bases: *const SvG1Affine, scalars: *const SvFe, offsets: *const u64,
                                 count: usize, form: c_int, out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_msm_batch_device(d_bases: *const SvG1Affine, d_scalars: *const SvFe, d_offsets: *const u64,
                                        count: usize, max_terms: usize, form: c_int, device: c_int,
                                        stream: *mut c_void, d_out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_table_create(bases: *const SvG1Affine, n: usize, form: c_int, device: c_int,
                                    handle: *mut u64) -> c_int;
    pub fn sv_bn254_g1_table_destroy(handle: u64) -> c_int;
    pub fn sv_bn254_g1_msm_batch_table(handle: u64, base_idx: *const u32, scalars: *const SvFe,
                                       offsets: *const u64, count: usize, form: c_int,
                                       out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_msm_batch_table_device(handle: u64, d_base_idx: *const u32, d_scalars: *const SvFe,
                                              d_offsets: *const u64, count: usize, form: c_int, stream: *mut c_void,
                                              d_out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_g1_table_device(handle: u64, device: *mut c_int) -> c_int;
    pub fn sv_bn254_g1_msm_batch_indexed_device(d_table: *const SvG1Affine, table_len: usize, table_form: c_int,
                                                d_base_idx: *const u32, d_scalars: *const SvFe,
                                                d_offsets: *const u64, count: usize, max_terms: usize,
                                                form: c_int, device: c_int, stream: *mut c_void,
                                                d_out: *mut SvG1Affine) -> c_int;
    pub fn sv_bn254_poseidon_permute(states: *mut SvFe, n: usize, t: c_int, form: c_int) -> c_int;
    pub fn sv_bn254_poseidon_permute_device(d_states: *mut SvFe, n: usize, t: c_int, form: c_int, device: c_int,
                                            stream: *mut c_void) -> c_int;
    pub fn sv_bn254_poseidon_squeeze(states: *mut SvFe, elements: *const SvFe, offsets: *const u64, n: usize,
                                     t: c_int, form: c_int, out: *mut SvFe) -> c_int;
    pub fn sv_bn254_poseidon_squeeze_device(d_states: *mut SvFe, d_elements: *const SvFe, d_offsets: *const u64,
                                            n: usize, t: c_int, form: c_int, d_out: *mut SvFe, device: c_int,
                                            stream: *mut c_void) -> c_int;
    pub fn sv_bn254_g1_decode(data: *const u8, n: usize, encoding: c_int, form: c_int, out: *mut SvG1Affine,
                              first_invalid: *mut i64) -> c_int;
    pub fn sv_bn254_g1_decode_device(d_data: *const u8, n: usize, encoding: c_int, form: c_int, device: c_int,
                                     stream: *mut c_void, d_out: *mut SvG1Affine, first_invalid: *mut i64) -> c_int;
    pub fn sv_bn254_kzg_accumulators_from_limbs(limbs: *const SvFe, n: usize, n_limbs: c_int, bits: c_int,
                                                form: c_int, lhs: *mut SvG1Affine, rhs: *mut SvG1Affine,
                                                first_invalid: *mut i64) -> c_int;
    pub fn sv_bn254_kzg_decide_eip197(input: *const u8, n_checks: usize, num_gpus: c_int,
                                      first_fail: *mut i32) -> c_int;
    pub fn sv_gen_scalars_device(d_scalars: *mut SvFe, n: usize, seed: u64, start: u64, form: c_int,
                                 device: c_int, stream: *mut c_void) -> c_int;
    pub fn sv_gen_bases_device(d_bases: *mut SvG1Affine, n: usize, seed: u64, start: u64, form: c_int,
                               device: c_int, stream: *mut c_void) -> c_int;
    pub fn sv_msm_last_stats(out: *mut SvMsmStats) -> c_int;
    pub fn sv_kzg_last_kernel_ms(out: *mut f32) -> c_int;
}

// halo2curves 0.3.1 keeps Fq / Fr as 4 x u64 little-endian Montgomery limbs and G1Affine as
// {x, y} (identity (0, 0)), G2Affine as {x: Fq2{c0, c1}, y}: byte-identical to the C structs.
const _: () = assert!(std::mem::size_of::<SvG1Affine>() == 64);
const _: () = assert!(std::mem::size_of::<SvG2Affine>() == 128);
const _: () = assert!(std::mem::size_of::<SvMsmRef>() == 16);

/// Message of this thread's last non-OK status.
pub fn last_error() -> String {
    unsafe {
        let p = sv_last_error();
        if p.is_null() { String::new() } else { std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned() }
    }
}

/// Smallest MSM routed to the GPU (SVGPU_MIN_MSM, default 2).  Measured on the MI355X box
/// (bench.py `verifier_msms.crossover`, profiles/r06_verifier_msms.json): one library call
/// (sv_bn254_g1_msm_refs: gather + copy + the small-MSM window path + host Horner) takes
/// 0.13-0.16 ms from 1 to 64 terms, the reference's naive CPU sum ~0.097 ms per term, so the GPU
/// wins from 2 terms -- a verifier's tens-term MSMs (bdfg21.rs:75-78) go to the GPU.
pub fn min_msm() -> usize {
    static INIT: Once = Once::new();
    static MIN: AtomicUsize = AtomicUsize::new(2);
    // call_once's completion happens-before every later return from it, so a relaxed load sees it
    INIT.call_once(|| {
        if let Some(v) = std::env::var("SVGPU_MIN_MSM").ok().and_then(|v| v.parse::<usize>().ok()) {
            MIN.store(v, Ordering::Relaxed);
        }
    });
    MIN.load(Ordering::Relaxed)
}

/// True when a GPU is usable, SVGPU_DISABLE is unset and halo2curves' memory layout is the one
/// the zero-copy calls assume (checked once, process-wide).
pub fn available() -> bool {
    static INIT: Once = Once::new();
    static READY: AtomicBool = AtomicBool::new(false);
    INIT.call_once(|| {
        if std::env::var_os("SVGPU_DISABLE").is_some() {
            return;
        }
        let layout_ok = std::mem::size_of::<G1Affine>() == 64
            && std::mem::size_of::<G2Affine>() == 128
            && std::mem::size_of::<Fr>() == 32
            && unsafe { std::mem::transmute::<Fq, [u64; 4]>(Fq::one()) }
                == [0xd35d438dc58f0d9d, 0x0a78eb28f5c70b3d, 0x666ea36f7879462c, 0x0e0a77c19a07df2f];
        READY.store(layout_ok && unsafe { sv_init(0) } == SV_OK, Ordering::Relaxed);
    });
    READY.load(Ordering::Relaxed)
}

/// Reinterpret a generic curve's slices as BN254 ones.  Both element types are checked at run
/// time (scalars must be `Fr`, bases `G1Affine`), so the cast is a no-op view of the same types
/// and the function is sound for any caller; it panics on any other pair of types.
pub fn cast_slices<'a, S: 'static, C: 'static>(scalars: &'a [S], bases: &'a [C]) -> (&'a [Fr], &'a [G1Affine]) {
    assert_eq!(std::any::TypeId::of::<S>(), std::any::TypeId::of::<Fr>(), "scalars are not bn256::Fr");
    assert_eq!(std::any::TypeId::of::<C>(), std::any::TypeId::of::<G1Affine>(), "bases are not bn256::G1Affine");
    // SAFETY: S == Fr and C == G1Affine (checked above): same type, same length, same lifetime
    unsafe {
        (std::slice::from_raw_parts(scalars.as_ptr() as *const Fr, scalars.len()),
         std::slice::from_raw_parts(bases.as_ptr() as *const G1Affine, bases.len()))
    }
}

/// The inverse cast of a BN254 result back to the caller's (identical) curve type.
pub fn cast_back<C: 'static + Copy>(p: G1Affine) -> C {
    assert_eq!(std::any::TypeId::of::<C>(), std::any::TypeId::of::<G1Affine>());
    unsafe { std::mem::transmute_copy::<G1Affine, C>(&p) }
}

fn g1_out(p: SvG1Affine) -> G1Affine {
    unsafe { std::mem::transmute::<SvG1Affine, G1Affine>(p) }
}

fn same_type<A: 'static, B: 'static>() -> bool {
    std::any::TypeId::of::<A>() == std::any::TypeId::of::<B>()
}

/// True when the pairing engine `M` is halo2curves' BN254 (`bn256::Bn256`): its G1 and G2 affine
/// types are `bn256::G1Affine` / `bn256::G2Affine`.  Needs no `M: 'static` bound (the decider's
/// `impl<M: MultiMillerLoop, MOS>` has none, pcs/kzg/decider.rs:53-57): the engine's affine types
/// are `PrimeCurveAffine`, which is `'static`.
pub fn is_bn256<M: Engine>() -> bool {
    same_type::<M::G1Affine, G1Affine>() && same_type::<M::G2Affine, G2Affine>()
}

/// `Some(&[bn256::G1Affine])` view of a generic curve's slice when `C` is `bn256::G1Affine`.
pub fn as_g1_slice<C: 'static>(points: &[C]) -> Option<&[G1Affine]> {
    // SAFETY: C == G1Affine (checked): same type, same length, same lifetime
    same_type::<C, G1Affine>()
        .then(|| unsafe { std::slice::from_raw_parts(points.as_ptr() as *const G1Affine, points.len()) })
}

/// `Some(&bn256::G2Affine)` view of a generic G2 point when `G` is `bn256::G2Affine`.
pub fn as_g2<G: 'static>(point: &G) -> Option<&G2Affine> {
    // SAFETY: G == G2Affine (checked)
    same_type::<G, G2Affine>().then(|| unsafe { &*(point as *const G as *const G2Affine) })
}

/// NativeLoader::multi_scalar_multiplication for a generic curve (loader/native.rs:61-71): the
/// call site passes its `&[(&C::Scalar, &C)]` unchanged.  `None` when `C` is not BN254 G1 (or its
/// scalar not `bn256::Fr`), when no GPU is usable, or on a device error; the caller then runs its
/// own CPU fold.  The `SvMsmRef`s are built straight from the generic pairs, so nothing is cast
/// unless both `TypeId`s match.  Panics on empty input like the reference (native.rs:69).
pub fn msm_generic<C: CurveAffine>(pairs: &[(&C::Scalar, &C)]) -> Option<C> {
    if pairs.is_empty() {
        panic!("pairs should not be empty");
    }
    if !(same_type::<C, G1Affine>() && same_type::<C::Scalar, Fr>()) || !available() {
        return None;
    }
    let refs: Vec<SvMsmRef> = pairs
        .iter()
        .map(|(s, b)| SvMsmRef { scalar: *s as *const C::Scalar as *const SvFe, base: *b as *const C as *const SvG1Affine })
        .collect();
    let mut out = SvG1Affine::default();
    let rc = unsafe { sv_bn254_g1_msm_refs(refs.as_ptr(), refs.len(), SV_MONTGOMERY, 0, &mut out) };
    (rc == SV_OK).then(|| cast_back::<C>(g1_out(out)))
}

/// decide_all for a generic engine's points (pcs/kzg/decider.rs:70-80): `dk.g2`, `dk.s_g2` and the
/// accumulators' `lhs`/`rhs` as the decider holds them (`M::G2Affine`, `M::G1Affine`).
/// `Some(-1)` = all pass, `Some(i)` = first failing accumulator (`try_collect` order), `None` =
/// not BN254, no GPU, or a device error (the caller keeps its sequential CPU decide).
pub fn decide_all_generic<G1: 'static, G2: 'static>(g2: &G2, s_g2: &G2, lhs: &[G1], rhs: &[G1]) -> Option<i32> {
    assert!(!lhs.is_empty());
    assert_eq!(lhs.len(), rhs.len());
    let (g2, s_g2) = (as_g2(g2)?, as_g2(s_g2)?);
    let (lhs, rhs) = (as_g1_slice(lhs)?, as_g1_slice(rhs)?);
    if !available() {
        return None;
    }
    decide_all(g2, s_g2, lhs, rhs)
}

/// NativeLoader::multi_scalar_multiplication (snark-verifier/src/loader/native.rs:61-71): the
/// pairs are passed as references; libsvgpu gathers them itself (pinned staging, host pool).
/// Panics on empty input like the reference (native.rs:69).  `None` = device error.
pub fn msm(pairs: &[(&Fr, &G1Affine)]) -> Option<G1Affine> {
    if pairs.is_empty() {
        panic!("pairs should not be empty");
    }
    // a Rust tuple's field order is unspecified: map explicitly (16 B per pair, sequential)
    let refs: Vec<SvMsmRef> = pairs
        .iter()
        .map(|(s, b)| SvMsmRef { scalar: *s as *const Fr as *const SvFe, base: *b as *const G1Affine as *const SvG1Affine })
        .collect();
    let mut out = SvG1Affine::default();
    let rc = unsafe { sv_bn254_g1_msm_refs(refs.as_ptr(), refs.len(), SV_MONTGOMERY, 0, &mut out) };
    (rc == SV_OK).then(|| g1_out(out))
}

/// util::msm::multi_scalar_multiplication (snark-verifier/src/util/msm.rs:287-316): contiguous
/// slices go zero-copy (halo2curves memory is the ABI's Montgomery layout).
pub fn msm_slices(scalars: &[Fr], bases: &[G1Affine]) -> Option<G1Affine> {
    assert_eq!(scalars.len(), bases.len());
    if bases.is_empty() {
        // the reference panics on an empty MSM: multi_scalar_multiplication_serial indexes
        // scalars[0] (msm.rs:244), reached with or without `parallel` (msm.rs:295-298, :313-314)
        panic!("index out of bounds: the len is 0 but the index is 0");
    }
    let mut out = SvG1Affine::default();
    let rc = unsafe {
        sv_bn254_g1_msm(bases.as_ptr() as *const SvG1Affine, scalars.as_ptr() as *const SvFe, bases.len(),
                        SV_MONTGOMERY, 0, &mut out)
    };
    (rc == SV_OK).then(|| g1_out(out))
}

/// AccumulationDecider::decide_all for KzgAs on NativeLoader (pcs/kzg/decider.rs:70-80):
/// Some(-1) = all pass, Some(i) = first failing accumulator, None = device error.
pub fn decide_all(g2: &G2Affine, s_g2: &G2Affine, lhs: &[G1Affine], rhs: &[G1Affine]) -> Option<i32> {
    assert!(!lhs.is_empty());
    assert_eq!(lhs.len(), rhs.len());
    let mut ff = -2i32;
    let rc = unsafe {
        sv_bn254_kzg_decide(g2 as *const G2Affine as *const SvG2Affine, s_g2 as *const G2Affine as *const SvG2Affine,
                            lhs.as_ptr() as *const SvG1Affine, rhs.as_ptr() as *const SvG1Affine, lhs.len(),
                            SV_MONTGOMERY, 0, &mut ff)
    };
    (rc == SV_OK).then_some(ff)
}

/// KzgAs::create_proof without blind (pcs/kzg/accumulation.rs:146-195): (Σ rⁱ lhsᵢ, Σ rⁱ rhsᵢ).
pub fn accumulate(lhs: &[G1Affine], rhs: &[G1Affine], r: &Fr) -> Option<(G1Affine, G1Affine)> {
    assert!(!lhs.is_empty());
    assert_eq!(lhs.len(), rhs.len());
    let (mut ol, mut or) = (SvG1Affine::default(), SvG1Affine::default());
    let rc = unsafe {
        sv_bn254_kzg_accumulate(lhs.as_ptr() as *const SvG1Affine, rhs.as_ptr() as *const SvG1Affine, lhs.len(),
                                r as *const Fr as *const SvFe, SV_MONTGOMERY, 0, &mut ol, &mut or)
    };
    (rc == SV_OK).then(|| (g1_out(ol), g1_out(or)))
}

/// KzgAs::create_proof without blind, challenge included (pcs/kzg/accumulation.rs:146-195): the
/// accumulators are absorbed into a Poseidon transcript (fresh when `sponge_state` is None, else
/// continuing from that state, which receives the state after the squeeze) and r is squeezed
/// (:158-176); returns (Σ rⁱ lhsᵢ, Σ rⁱ rhsᵢ, r).  `Err(true)` = an identity accumulator point,
/// which the reference reports as `Error::Transcript` ("Invalid elliptic curve point encoding in
/// proof", transcript/halo2.rs:214-226).  `Err(false)` = anything else the library refused: a
/// device error, or an argument error that is not the identity case (an unreduced coordinate or
/// sponge-state element); the caller then keeps its own CPU path, which reports such input itself.
pub fn create_proof(lhs: &[G1Affine], rhs: &[G1Affine], sponge_state: Option<&mut [Fr; 3]>)
                    -> Result<(G1Affine, G1Affine, Fr), bool> {
    assert!(!lhs.is_empty());
    assert_eq!(lhs.len(), rhs.len());
    let (mut ol, mut or) = (SvG1Affine::default(), SvG1Affine::default());
    let mut r = Fr::zero();
    let st = sponge_state.map_or(std::ptr::null_mut(), |s| s.as_mut_ptr() as *mut SvFe);
    let rc = unsafe {
        sv_bn254_kzg_create_proof(lhs.as_ptr() as *const SvG1Affine, rhs.as_ptr() as *const SvG1Affine, lhs.len(),
                                  SV_MONTGOMERY, 0, &mut ol, &mut or, st, &mut r as *mut Fr as *mut SvFe)
    };
    match rc {
        SV_OK => Ok((g1_out(ol), g1_out(or), r)),
        SV_ERR_ARG if last_error().starts_with(IDENTITY_MSG) => Err(true),
        _ => Err(false),
    }
}

/// Prefix of `sv_last_error()` for an identity accumulator point (csrc/api.cpp), the reference's
/// Error::Transcript message.
pub const IDENTITY_MSG: &str = "Invalid elliptic curve point encoding in proof";

/// Many small MSMs in one launch: MSM k = terms offsets[k]..offsets[k+1].
pub fn msm_batch(scalars: &[Fr], bases: &[G1Affine], offsets: &[u64]) -> Option<Vec<G1Affine>> {
    assert_eq!(scalars.len(), bases.len());
    let count = offsets.len().saturating_sub(1);
    let mut out = vec![SvG1Affine::default(); count];
    let rc = unsafe {
        sv_bn254_g1_msm_batch(bases.as_ptr() as *const SvG1Affine, scalars.as_ptr() as *const SvFe,
                              offsets.as_ptr(), count, SV_MONTGOMERY, out.as_mut_ptr())
    };
    if rc == SV_ERR_EMPTY {
        panic!("pairs should not be empty");
    }
    (rc == SV_OK).then(|| out.into_iter().map(g1_out).collect())
}

/// Device-resident constant bases (Protocol::loaded, plonk/protocol.rs:106-131), uploaded once.
pub struct BaseTable {
    handle: u64,
}

impl BaseTable {
    pub fn new(bases: &[G1Affine], device: i32) -> Option<Self> {
        let mut handle = 0u64;
        let rc = unsafe {
            sv_bn254_g1_table_create(bases.as_ptr() as *const SvG1Affine, bases.len(), SV_MONTGOMERY, device,
                                     &mut handle)
        };
        (rc == SV_OK).then_some(BaseTable { handle })
    }

    /// MSM k = Σ scalars[i] · table[base_idx[i]] over i in offsets[k]..offsets[k+1].
    pub fn msm_batch(&self, base_idx: &[u32], scalars: &[Fr], offsets: &[u64]) -> Option<Vec<G1Affine>> {
        assert_eq!(base_idx.len(), scalars.len());
        let count = offsets.len().saturating_sub(1);
        let mut out = vec![SvG1Affine::default(); count];
        let rc = unsafe {
            sv_bn254_g1_msm_batch_table(self.handle, base_idx.as_ptr(), scalars.as_ptr() as *const SvFe,
                                        offsets.as_ptr(), count, SV_MONTGOMERY, out.as_mut_ptr())
        };
        if rc == SV_ERR_EMPTY {
            panic!("pairs should not be empty");
        }
        (rc == SV_OK).then(|| out.into_iter().map(g1_out).collect())
    }
}

impl Drop for BaseTable {
    fn drop(&mut self) {
        unsafe {
            sv_bn254_g1_table_destroy(self.handle);
        }
    }
}

/// Poseidon::squeeze (util/hash/poseidon.rs:455-467) on a batch of sponges (one per transcript):
/// states (n x t, Montgomery Fr, in/out) and each sponge's buffered input elements[offsets[j]..].
pub fn poseidon_squeeze(states: &mut [Fr], elements: &[Fr], offsets: &[u64], t: usize) -> Option<Vec<Fr>> {
    let n = offsets.len().saturating_sub(1);
    assert_eq!(states.len(), n * t);
    let mut out = vec![Fr::zero(); n];
    let rc = unsafe {
        sv_bn254_poseidon_squeeze(states.as_mut_ptr() as *mut SvFe, elements.as_ptr() as *const SvFe,
                                  offsets.as_ptr(), n, t as c_int, SV_MONTGOMERY, out.as_mut_ptr() as *mut SvFe)
    };
    (rc == SV_OK).then_some(out)
}

/// read_ec_point for a whole proof (transcript/halo2.rs:247-260 compressed, transcript/evm.rs:223-242
/// EVM): Ok(points), Err(Some(i)) = first invalid encoding (the reference's Error::Transcript),
/// Err(None) = device error.
pub fn decode_points(data: &[u8], encoding: c_int) -> Result<Vec<G1Affine>, Option<usize>> {
    let rec = if encoding == SV_ENC_EVM { 64 } else { 32 };
    let n = data.len() / rec;
    let mut out = vec![SvG1Affine::default(); n];
    let mut first_invalid = -1i64;
    let rc = unsafe { sv_bn254_g1_decode(data.as_ptr(), n, encoding, SV_MONTGOMERY, out.as_mut_ptr(), &mut first_invalid) };
    match rc {
        SV_OK => Ok(out.into_iter().map(g1_out).collect()),
        SV_ERR_ARG if first_invalid >= 0 => Err(Some(first_invalid as usize)),
        _ => Err(None),
    }
}

/// LimbsEncoding::from_repr (pcs/kzg/accumulator.rs:57-77) for many accumulators at once.
pub fn accumulators_from_limbs(limbs: &[Fr], n_limbs: usize, bits: usize)
                               -> Result<Vec<(G1Affine, G1Affine)>, Option<usize>> {
    let n = limbs.len() / (4 * n_limbs);
    let (mut l, mut r) = (vec![SvG1Affine::default(); n], vec![SvG1Affine::default(); n]);
    let mut first_invalid = -1i64;
    let rc = unsafe {
        sv_bn254_kzg_accumulators_from_limbs(limbs.as_ptr() as *const SvFe, n, n_limbs as c_int, bits as c_int,
                                             SV_MONTGOMERY, l.as_mut_ptr(), r.as_mut_ptr(), &mut first_invalid)
    };
    match rc {
        SV_OK => Ok(l.into_iter().map(g1_out).zip(r.into_iter().map(g1_out)).collect()),
        SV_ERR_ARG if first_invalid >= 0 => Err(Some(first_invalid as usize)),
        _ => Err(None),
    }
}

/// A batch of EIP-197 ecPairing inputs as the EVM decider lays them out (decider.rs:107-127).
pub fn decide_eip197(input: &[u8]) -> Option<i32> {
    assert_eq!(input.len() % 0x180, 0);
    let mut ff = -2i32;
    let rc = unsafe { sv_bn254_kzg_decide_eip197(input.as_ptr(), input.len() / 0x180, 0, &mut ff) };
    (rc == SV_OK).then_some(ff)
}
