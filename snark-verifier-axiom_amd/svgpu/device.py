"""Device-resident (HBM) entry points over torch tensors.

PyTorch is plumbing here: it owns device memory and the stream; the work is libsvgpu's HIP
kernels.  Tensors are int64 views of the C-ABI layouts: bases (n, 8), scalars (n, 4).
"""
from __future__ import annotations

import copy
import ctypes
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from . import encoding as enc


def _stream_handle(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _dev_index(t: torch.Tensor) -> int:
    if t.device.type != "cuda":
        raise _lib.DeviceError("tensor must live on a GPU (cuda/HIP device)")
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def empty_bases(n: int, device) -> torch.Tensor:
    return torch.empty((n, 8), dtype=torch.int64, device=device)


def empty_scalars(n: int, device) -> torch.Tensor:
    return torch.empty((n, 4), dtype=torch.int64, device=device)


def gen_bases(t: torch.Tensor, seed: int, start: int = 0, form: int = _lib.SV_MONTGOMERY) -> torch.Tensor:
    d = _dev_index(t)
    _lib.check(_lib.lib.sv_gen_bases_device(t.data_ptr(), t.shape[0], seed, start, form, d,
                                            _stream_handle(t.device)), "sv_gen_bases_device")
    return t


def gen_scalars(t: torch.Tensor, seed: int, start: int = 0, form: int = _lib.SV_MONTGOMERY) -> torch.Tensor:
    d = _dev_index(t)
    _lib.check(_lib.lib.sv_gen_scalars_device(t.data_ptr(), t.shape[0], seed, start, form, d,
                                              _stream_handle(t.device)), "sv_gen_scalars_device")
    return t


def msm_partial(bases: torch.Tensor, scalars: torch.Tensor, form: int = _lib.SV_MONTGOMERY) -> Tuple[int, int, int]:
    """One device's MSM over HBM-resident inputs -> canonical Jacobian (X, Y, Z) on the host."""
    if bases.shape[0] != scalars.shape[0]:
        raise ValueError("bases and scalars differ in length")
    d = _dev_index(bases)
    out = _lib.sv_g1_jacobian()
    _lib.check(_lib.lib.sv_bn254_g1_msm_device(bases.data_ptr(), scalars.data_ptr(), bases.shape[0], form, d,
                                               _stream_handle(bases.device), ctypes.byref(out)),
               "sv_bn254_g1_msm_device")
    return enc.jacobian_from_struct(out)


def msm(bases: torch.Tensor, scalars: torch.Tensor, form: int = _lib.SV_MONTGOMERY):
    """One device's MSM -> affine point (canonical ints; None = identity).  The Jacobian partial
    goes straight from sv_bn254_g1_msm_device into sv_bn254_g1_fold (no Python-int round trip)."""
    if bases.shape[0] != scalars.shape[0]:
        raise ValueError("bases and scalars differ in length")
    d = _dev_index(bases)
    part = _lib.sv_g1_jacobian()
    _lib.check(_lib.lib.sv_bn254_g1_msm_device(bases.data_ptr(), scalars.data_ptr(), bases.shape[0], form, d,
                                               _stream_handle(bases.device), ctypes.byref(part)),
               "sv_bn254_g1_msm_device")
    out = _lib.sv_g1_affine()
    _lib.check(_lib.lib.sv_bn254_g1_fold(ctypes.byref(part), 1, ctypes.byref(out), _lib.SV_CANONICAL),
               "sv_bn254_g1_fold")
    return enc.g1_from_struct(out)


def last_msm_stats() -> dict:
    s = _lib.sv_msm_stats()
    _lib.check(_lib.lib.sv_msm_last_stats(ctypes.byref(s)), "sv_msm_last_stats")
    return {name: getattr(s, name) for name, _ in s._fields_}


def decide(g2, s_g2, lhs: torch.Tensor, rhs: torch.Tensor, form: int = _lib.SV_CANONICAL,
           want_gt: bool = False) -> Tuple[int, List[int], Optional[List[List[int]]]]:
    """Decider over HBM-resident accumulators -> (first_fail, verdicts, Gt values or None)."""
    n = lhs.shape[0]
    d = _dev_index(lhs)
    ff = ctypes.c_int32(-2)
    # numpy buffer + tolist(): 256 verdicts in ~5 us where list() of a ctypes array took ~15 us
    verdicts = np.empty(n, dtype=np.int32)
    gt = (_lib.sv_fq12 * n)() if want_gt else None
    g2s, sg2s = _g2_struct_cached(g2, form), _g2_struct_cached(s_g2, form)
    _lib.check(_lib.lib.sv_bn254_kzg_decide_device(
        ctypes.byref(g2s), ctypes.byref(sg2s), lhs.data_ptr(), rhs.data_ptr(), n, form, d,
        _stream_handle(lhs.device), ctypes.byref(ff), verdicts.ctypes.data,
        ctypes.cast(gt, ctypes.c_void_p) if gt is not None else None), "sv_bn254_kzg_decide_device")
    gts = [enc.fq12_from_struct(g) for g in gt] if gt is not None else None
    return ff.value, verdicts.tolist(), gts


_G2_CACHE: dict = {}
# The same key object passed again (the usual verifier loop): (id, form) -> (object, a deep copy of
# it, struct).  A hit needs the very object AND equal contents (a C-level compare, ~0.1 us), so a
# list mutated in place misses; the content-keyed _G2_CACHE below costs ~2.7 us (Python freezing).
_G2_RECENT: dict = {}


def _frozen(v):
    """Nested lists (a G2 point as ((x0, x1), (y0, y1)) in any sequence type) as nested tuples."""
    return tuple(_frozen(x) for x in v) if isinstance(v, (list, tuple)) else v


def _g2_struct_cached(q, form: int):
    """A deciding key's G2 point as its ABI struct, converted once per key (a verifier decides with
    one key over and over; the library only reads the struct during the call)."""
    plain = type(q) in (list, tuple)
    if plain:
        e = _G2_RECENT.get((id(q), form))
        try:
            if e is not None and e[0] is q and bool(e[1] == q):
                return e[2]
        except (TypeError, ValueError):  # elements whose == is not a plain bool (arrays): no fast path
            plain = False
    try:
        key = (_frozen(q), form)
        hash(key)
    except TypeError:  # something hash cannot take even after freezing: no caching
        return enc.g2_struct(q, form)
    s = _G2_CACHE.get(key)
    if s is None:
        if len(_G2_CACHE) >= 16:
            _G2_CACHE.clear()
        s = _G2_CACHE[key] = enc.g2_struct(q, form)
    if plain:
        if len(_G2_RECENT) >= 16:
            _G2_RECENT.clear()
        _G2_RECENT[(id(q), form)] = (q, copy.deepcopy(q), s)
    return s


def last_decide_kernel_ms() -> float:
    """Kernel time of this thread's last decider launch (HIP events on the call's stream)."""
    v = ctypes.c_float(0)
    _lib.check(_lib.lib.sv_kzg_last_kernel_ms(ctypes.byref(v)), "sv_kzg_last_kernel_ms")
    return float(v.value)


def poseidon_squeeze(states: torch.Tensor, elements: torch.Tensor, offsets: torch.Tensor, t: int = 3,
                     form: int = _lib.SV_MONTGOMERY, out: torch.Tensor = None) -> torch.Tensor:
    """Poseidon::squeeze on n HBM-resident sponges (states: (n * t, 4) int64 limbs, in/out;
    elements: (m, 4); offsets: (n + 1,) int64, sponge j absorbs elements[offsets[j]:offsets[j+1]]).
    Returns out (n, 4): the challenges."""
    n = offsets.shape[0] - 1
    if states.shape[0] != n * t:
        raise _lib.LengthError(f"poseidon: {states.shape[0]} state rows for {n} sponges of width {t}")
    if out is None:
        out = torch.empty((max(n, 1), 4), dtype=torch.int64, device=states.device)
    d = _dev_index(states)
    _lib.check(_lib.lib.sv_bn254_poseidon_squeeze_device(states.data_ptr(), elements.data_ptr(), offsets.data_ptr(),
                                                         n, t, form, out.data_ptr(), d,
                                                         _stream_handle(states.device)),
               "sv_bn254_poseidon_squeeze_device")
    return out[:n]


def poseidon_permute(states: torch.Tensor, t: int = 3, form: int = _lib.SV_MONTGOMERY) -> torch.Tensor:
    """In-place HADES permutation of (n * t, 4) HBM-resident states."""
    d = _dev_index(states)
    _lib.check(_lib.lib.sv_bn254_poseidon_permute_device(states.data_ptr(), states.shape[0] // t, t, form, d,
                                                         _stream_handle(states.device)),
               "sv_bn254_poseidon_permute_device")
    return states


def msm_batch(bases: torch.Tensor, scalars: torch.Tensor, offsets: torch.Tensor, max_terms: int,
              form: int = _lib.SV_MONTGOMERY, out: torch.Tensor = None) -> torch.Tensor:
    """Batched MSMs over HBM-resident arrays (offsets: (count + 1,) int64 on the device);
    returns (count, 8) int64 affine results in `form`."""
    count = offsets.shape[0] - 1
    if out is None:
        out = torch.empty((max(count, 1), 8), dtype=torch.int64, device=bases.device)
    d = _dev_index(bases)
    _lib.check(_lib.lib.sv_bn254_g1_msm_batch_device(bases.data_ptr(), scalars.data_ptr(), offsets.data_ptr(),
                                                     count, max_terms, form, d, _stream_handle(bases.device),
                                                     out.data_ptr()),
               "sv_bn254_g1_msm_batch_device")
    return out[:count]


def msm_batch_indexed(table: torch.Tensor, base_idx: torch.Tensor, scalars: torch.Tensor, offsets: torch.Tensor,
                      max_terms: int, form: int = _lib.SV_MONTGOMERY, table_form: int = _lib.SV_MONTGOMERY,
                      out: torch.Tensor = None) -> torch.Tensor:
    """Batched MSMs whose terms reference rows of an HBM-resident base table (table: (rows, 8) int64;
    base_idx: (terms,) int32 row indices; offsets: (count + 1,) int64); returns (count, 8) int64."""
    count = offsets.shape[0] - 1
    if out is None:
        out = torch.empty((max(count, 1), 8), dtype=torch.int64, device=scalars.device)
    d = _dev_index(scalars)
    _lib.check(_lib.lib.sv_bn254_g1_msm_batch_indexed_device(table.data_ptr(), table.shape[0], table_form,
                                                             base_idx.data_ptr(), scalars.data_ptr(),
                                                             offsets.data_ptr(), count, max_terms, form, d,
                                                             _stream_handle(scalars.device), out.data_ptr()),
               "sv_bn254_g1_msm_batch_indexed_device")
    return out[:count]
