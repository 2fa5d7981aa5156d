"""Host-side mirror of the reference's MSM entry points, executed by libsvgpu on the GPU.

* ``NativeLoader.multi_scalar_multiplication(pairs)`` mirrors
  ``EcPointLoader::multi_scalar_multiplication`` for ``NativeLoader``
  (snark-verifier/src/loader/native.rs:61-71): sum of ``base * scalar`` over the pairs, as an
  affine point; empty input panics with "pairs should not be empty" (native.rs:69).
* ``multi_scalar_multiplication(scalars, bases)`` mirrors ``util::msm::multi_scalar_multiplication``
  (snark-verifier/src/util/msm.rs:287-316), whose length check is ``assert_eq!`` (msm.rs:288).

* ``batch_multi_scalar_multiplication(msms)`` / ``NativeLoader.multi_scalar_multiplication_batch``
  evaluate many such MSMs in one call (the per-proof Msm::evaluate calls of a
  native verifier, bdfg21.rs:75-78 / gwc19.rs:76-79, and accumulation.rs:177-192's pair).

Points are ``(x, y)`` tuples of canonical ints, ``None`` is the identity (halo2curves (0, 0)).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from . import encoding as enc

Point = Optional[Tuple[int, int]]


class ReferencePanic(AssertionError):
    """A condition under which the Rust reference panics."""


def msm_arrays(bases: np.ndarray, scalars: np.ndarray, form: int = _lib.SV_CANONICAL, num_gpus: int = 0) -> Point:
    """MSM over C-ABI-layout host arrays: bases (n, 8) u64, scalars (n, 4) u64."""
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
    if bases.shape[0] != scalars.shape[0]:
        raise ReferencePanic("assertion failed: scalars.len() == bases.len()")
    out = _lib.sv_g1_affine()
    rc = _lib.lib.sv_bn254_g1_msm(bases.ctypes.data, scalars.ctypes.data, bases.shape[0], form, num_gpus,
                                  ctypes.byref(out))
    if rc == _lib.SV_ERR_EMPTY:
        raise ReferencePanic("pairs should not be empty")
    _lib.check(rc, "sv_bn254_g1_msm")
    return enc.g1_from_struct(out, form)


def make_refs(scalar_ptrs: np.ndarray, base_ptrs: np.ndarray) -> np.ndarray:
    """Pack two equal-length arrays of host addresses (scalar_ptrs[i] -> sv_fe, base_ptrs[i] ->
    sv_g1_affine) into the (n, 2) u64 sv_msm_ref array of the C ABI."""
    sp = np.ascontiguousarray(scalar_ptrs, dtype=np.uint64)
    bp = np.ascontiguousarray(base_ptrs, dtype=np.uint64)
    if sp.shape != bp.shape:
        raise ReferencePanic("assertion failed: scalars.len() == bases.len()")
    return np.stack([sp, bp], axis=1)


def msm_refs(refs: np.ndarray, form: int = _lib.SV_CANONICAL, num_gpus: int = 0) -> Point:
    """MSM over references (the NativeLoader pairs shape, native.rs:61-71): `refs` is the (n, 2)
    u64 sv_msm_ref array (see make_refs); the library gathers the referenced values."""
    refs = np.ascontiguousarray(refs, dtype=np.uint64).reshape(-1, 2)
    out = _lib.sv_g1_affine()
    rc = _lib.lib.sv_bn254_g1_msm_refs(refs.ctypes.data, refs.shape[0], form, num_gpus, ctypes.byref(out))
    if rc == _lib.SV_ERR_EMPTY:
        raise ReferencePanic("pairs should not be empty")
    _lib.check(rc, "sv_bn254_g1_msm_refs")
    return enc.g1_from_struct(out, form)


def multi_scalar_multiplication(scalars: Sequence[int], bases: Sequence[Point], num_gpus: int = 0) -> Point:
    if len(scalars) != len(bases):
        raise ReferencePanic("assertion failed: scalars.len() == bases.len()")
    return msm_arrays(enc.bases_array(bases), enc.scalars_array(scalars), _lib.SV_CANONICAL, num_gpus)


def msm_batch_arrays(bases: np.ndarray, scalars: np.ndarray, offsets: Sequence[int],
                     form: int = _lib.SV_CANONICAL) -> list:
    """len(offsets) - 1 MSMs over shared C-ABI host arrays; MSM k uses rows offsets[k]:offsets[k+1]."""
    bases = np.ascontiguousarray(bases, dtype=np.uint64)
    scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
    if bases.shape[0] != scalars.shape[0]:
        raise ReferencePanic("assertion failed: scalars.len() == bases.len()")
    off = np.ascontiguousarray(offsets, dtype=np.uint64)
    count = off.shape[0] - 1
    if count <= 0:
        return []
    if int(off[-1]) > bases.shape[0]:
        raise _lib.LengthError("msm_batch: offsets run past the arrays")
    out = (_lib.sv_g1_affine * count)()
    rc = _lib.lib.sv_bn254_g1_msm_batch(bases.ctypes.data, scalars.ctypes.data, off.ctypes.data, count, form,
                                        ctypes.cast(out, ctypes.c_void_p))
    if rc == _lib.SV_ERR_EMPTY:
        raise ReferencePanic("pairs should not be empty")
    _lib.check(rc, "sv_bn254_g1_msm_batch")
    return [enc.g1_from_struct(o, form) for o in out]


class BaseTable:
    """Device-resident fixed bases (the generator and a circuit's preprocessed commitments, loaded
    once per verifier: Protocol::loaded, plonk/protocol.rs:106-131) referenced by row index from
    each proof's MSMs (Msm::evaluate, bdfg21.rs:75-78 / gwc19.rs:76-79), so a per-proof batch ships
    only scalars and u32 indices.  Rows are uploaded once in Montgomery form on `device` and expanded
    there to their window multiples 2^(8 w) P, so every batch runs in one bucket set per MSM with
    no window Horner (csrc/msm_batch.hip k_msm_batch_fixed)."""

    def __init__(self, bases, device: int = 0):
        if not isinstance(bases, np.ndarray):
            bases = enc.bases_array(list(bases))
        arr = np.ascontiguousarray(bases, dtype=np.uint64)
        self.n = arr.shape[0]
        self.handle = None
        h = ctypes.c_uint64(0)
        _lib.check(_lib.lib.sv_bn254_g1_table_create(arr.ctypes.data, self.n, _lib.SV_CANONICAL, device,
                                                     ctypes.byref(h)), "sv_bn254_g1_table_create")
        self.handle = h.value

    def close(self):
        if self.handle is not None:
            h, self.handle = self.handle, None
            _lib.check(_lib.lib.sv_bn254_g1_table_destroy(h), "sv_bn254_g1_table_destroy")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def msm_batch_arrays(self, base_idx: np.ndarray, scalars: np.ndarray, offsets: Sequence[int],
                         form: int = _lib.SV_CANONICAL) -> list:
        """MSM k = sum over i in [offsets[k], offsets[k+1]) of scalars[i] * table[base_idx[i]]."""
        if self.handle is None:
            raise _lib.ArgumentError("base table is closed")
        idx = np.ascontiguousarray(base_idx, dtype=np.uint32)
        scalars = np.ascontiguousarray(scalars, dtype=np.uint64)
        if idx.shape[0] != scalars.shape[0]:
            raise ReferencePanic("assertion failed: scalars.len() == bases.len()")
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        count = off.shape[0] - 1
        if count <= 0:
            return []
        if int(off[-1]) > idx.shape[0]:
            raise _lib.LengthError("msm_batch: offsets run past the arrays")
        out = (_lib.sv_g1_affine * count)()
        rc = _lib.lib.sv_bn254_g1_msm_batch_table(self.handle, idx.ctypes.data, scalars.ctypes.data,
                                                  off.ctypes.data, count, form, ctypes.cast(out, ctypes.c_void_p))
        if rc == _lib.SV_ERR_EMPTY:
            raise ReferencePanic("pairs should not be empty")
        _lib.check(rc, "sv_bn254_g1_msm_batch_table")
        return [enc.g1_from_struct(o, form) for o in out]

    def device(self) -> int:
        d = ctypes.c_int(-1)
        _lib.check(_lib.lib.sv_bn254_g1_table_device(self.handle, ctypes.byref(d)), "sv_bn254_g1_table_device")
        return d.value

    def msm_batch_device(self, base_idx, scalars, offsets, form: int = _lib.SV_MONTGOMERY, out=None):
        """HBM-resident form (torch tensors on the table's device): base_idx (terms,) int32, scalars
        (terms, 4) int64, offsets (count + 1,) int64 -> (count, 8) int64 affine results in `form`."""
        import torch
        if self.handle is None:
            raise _lib.ArgumentError("base table is closed")
        count = offsets.shape[0] - 1
        if out is None:
            out = torch.empty((max(count, 1), 8), dtype=torch.int64, device=scalars.device)
        stream = torch.cuda.current_stream(scalars.device).cuda_stream
        _lib.check(_lib.lib.sv_bn254_g1_msm_batch_table_device(self.handle, base_idx.data_ptr(), scalars.data_ptr(),
                                                                offsets.data_ptr(), count, form, stream,
                                                                out.data_ptr()), "sv_bn254_g1_msm_batch_table_device")
        return out[:count]

    def batch_multi_scalar_multiplication(self, msms: Sequence[Sequence[Tuple[int, int]]]) -> list:
        """msms: per MSM a list of (scalar, table row) pairs."""
        offsets = [0]
        scalars, idx = [], []
        for pairs in msms:
            if len(pairs) == 0:
                raise ReferencePanic("pairs should not be empty")
            scalars += [s for s, _ in pairs]
            idx += [i for _, i in pairs]
            offsets.append(len(scalars))
        if not msms:
            return []
        return self.msm_batch_arrays(np.array(idx, dtype=np.uint32), enc.scalars_array(scalars), offsets)


def batch_multi_scalar_multiplication(msms: Sequence[Sequence[Tuple[int, Point]]]) -> list:
    """[NativeLoader.multi_scalar_multiplication(pairs) for pairs in msms], one GPU launch."""
    offsets = [0]
    scalars, bases = [], []
    for pairs in msms:
        if len(pairs) == 0:
            raise ReferencePanic("pairs should not be empty")
        scalars += [s for s, _ in pairs]
        bases += [b for _, b in pairs]
        offsets.append(len(scalars))
    if not msms:
        return []
    return msm_batch_arrays(enc.bases_array(bases), enc.scalars_array(scalars), offsets)


class NativeLoader:
    """Mirror of snark_verifier::loader::native::NativeLoader (stateless, like the reference's
    ``lazy_static`` LOADER, native.rs:11-19)."""

    @staticmethod
    def multi_scalar_multiplication(pairs: Sequence[Tuple[int, Point]], num_gpus: int = 0) -> Point:
        if len(pairs) == 0:
            raise ReferencePanic("pairs should not be empty")
        scalars = [s for s, _ in pairs]
        bases = [b for _, b in pairs]
        return multi_scalar_multiplication(scalars, bases, num_gpus)

    @staticmethod
    def multi_scalar_multiplication_batch(msms: Sequence[Sequence[Tuple[int, Point]]]) -> list:
        return batch_multi_scalar_multiplication(msms)


def fold_partials(partials: Sequence[Tuple[int, int, int]], out_form: int = _lib.SV_CANONICAL) -> Point:
    """Fold canonical Jacobian partials (X, Y, Z) in order -> affine (host-only, no GPU)."""
    arr = (_lib.sv_g1_jacobian * len(partials))(*[enc.jacobian_struct(*p) for p in partials])
    out = _lib.sv_g1_affine()
    _lib.check(_lib.lib.sv_bn254_g1_fold(ctypes.cast(arr, ctypes.c_void_p), len(partials), ctypes.byref(out),
                                         out_form), "sv_bn254_g1_fold")
    return enc.g1_from_struct(out, out_form)
