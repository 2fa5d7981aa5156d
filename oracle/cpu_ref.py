"""ctypes wrapper of oracle/build/liboracle_bn254.so (C++ CPU restatement) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ (full-size parity on the GPU box), __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Build: ``make -C oracle/cpu``.  Arrays use the C-ABI layout (canonical limbs).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import c_int, c_int32, c_size_t, c_uint64, c_void_p

import numpy as np

LIB_PATH = os.environ.get("ORACLE_LIB",
                          os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "liboracle_bn254.so"))
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run `make -C oracle/cpu`")
        L = ctypes.CDLL(LIB_PATH)
        L.or_num_threads_default.restype = c_int
        L.or_msm_naive.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p]
        L.or_msm_pippenger.argtypes = [c_void_p, c_void_p, c_size_t, c_int, c_void_p]
        L.or_decide_all.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                    ctypes.POINTER(c_int32), c_void_p]
        L.or_count_decide_fpmul.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p]
        L.or_count_decide_fpmul.restype = c_uint64
        L.or_count_decide_fpmul_h2c.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        L.or_count_decide_fpmul_h2c.restype = c_uint64
        L.or_count_h2c_prepare.argtypes = [c_void_p, c_void_p]
        L.or_count_h2c_prepare.restype = c_uint64
        L.or_accumulate.argtypes = [c_void_p, c_void_p, c_size_t, c_void_p, c_void_p, c_void_p]
        L.or_gen_scalars.argtypes = [c_uint64, c_uint64, c_size_t, c_void_p]
        L.or_gen_scalars.restype = None
        L.or_gen_bases.argtypes = [c_uint64, c_uint64, c_size_t, c_int, c_void_p]
        L.or_gen_bases.restype = None
        _lib = L
    return _lib


def _c(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def default_threads() -> int:
    return lib().or_num_threads_default()


def msm_naive(bases, scalars) -> np.ndarray:
    bases, scalars = _c(bases), _c(scalars)
    out = np.zeros(8, dtype=np.uint64)
    if lib().or_msm_naive(bases.ctypes.data, scalars.ctypes.data, bases.shape[0], out.ctypes.data):
        raise AssertionError("pairs should not be empty")
    return out


def msm_pippenger(bases, scalars, threads: int = 0) -> np.ndarray:
    bases, scalars = _c(bases), _c(scalars)
    out = np.zeros(8, dtype=np.uint64)
    lib().or_msm_pippenger(bases.ctypes.data, scalars.ctypes.data, bases.shape[0], threads, out.ctypes.data)
    return out


def decide_all(g2: np.ndarray, s_g2: np.ndarray, lhs, rhs, threads: int = 1, want_gt: bool = False):
    g2, s_g2, lhs, rhs = _c(g2), _c(s_g2), _c(lhs), _c(rhs)
    n = lhs.shape[0]
    ff = c_int32(-2)
    gt = np.zeros((n, 48), dtype=np.uint64) if want_gt else None
    if lib().or_decide_all(g2.ctypes.data, s_g2.ctypes.data, lhs.ctypes.data, rhs.ctypes.data, n, threads,
                           ctypes.byref(ff), gt.ctypes.data if gt is not None else None):
        raise AssertionError("assertion failed: !accumulators.is_empty()")
    return ff.value, gt


def count_decide_fpmul(g2: np.ndarray, s_g2: np.ndarray, lhs_row, rhs_row) -> int:
    """Fq multiplications of one decide as restated in bn254_ref.cpp (decider roofline)."""
    g2, s_g2, l, r = _c(g2), _c(s_g2), _c(lhs_row), _c(rhs_row)
    return int(lib().or_count_decide_fpmul(g2.ctypes.data, s_g2.ctypes.data, l.ctypes.data, r.ctypes.data))


def count_decide_fpmul_h2c(g2: np.ndarray, s_g2: np.ndarray, lhs_row, rhs_row):
    """(Fq products, Gt value) of one decide in the halo2curves-structured restatement of
    bn254_ref.cpp (namespace h2c): the decider roofline's work unit, counted."""
    g2, s_g2, l, r = _c(g2), _c(s_g2), _c(lhs_row), _c(rhs_row)
    gt = np.zeros(48, dtype=np.uint64)
    n = int(lib().or_count_decide_fpmul_h2c(g2.ctypes.data, s_g2.ctypes.data, l.ctypes.data, r.ctypes.data,
                                            gt.ctypes.data))
    return n, gt


def count_h2c_prepare(g2: np.ndarray, s_g2: np.ndarray) -> int:
    """The Fq products of count_decide_fpmul_h2c spent in the two G2 line preparations
    (G2Prepared::from inside decide, decider.rs:64), which the GPU decider caches per key."""
    g2, s_g2 = _c(g2), _c(s_g2)
    return int(lib().or_count_h2c_prepare(g2.ctypes.data, s_g2.ctypes.data))


def accumulate(lhs, rhs, r: np.ndarray):
    lhs, rhs, r = _c(lhs), _c(rhs), _c(r)
    ol, orr = np.zeros(8, dtype=np.uint64), np.zeros(8, dtype=np.uint64)
    if lib().or_accumulate(lhs.ctypes.data, rhs.ctypes.data, lhs.shape[0], r.ctypes.data, ol.ctypes.data,
                           orr.ctypes.data):
        raise AssertionError("assertion failed: !instances.is_empty()")
    return ol, orr


def gen_scalars(seed: int, n: int, start: int = 0) -> np.ndarray:
    out = np.zeros((n, 4), dtype=np.uint64)
    lib().or_gen_scalars(seed, start, n, out.ctypes.data)
    return out


def gen_bases(seed: int, n: int, start: int = 0, threads: int = 0) -> np.ndarray:
    out = np.zeros((n, 8), dtype=np.uint64)
    lib().or_gen_bases(seed, start, n, threads or default_threads(), out.ctypes.data)
    return out
