"""ctypes binding of libsvgpu.so (include/svgpu.h).

The library is built in-tree (``make -C snark-verifier-axiom_amd`` -> ``build/libsvgpu.so``).
There is no fallback: if the shared object is missing this module raises at import time, and
compute calls without a GPU raise :class:`DeviceError` (status SV_ERR_DEVICE).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_int32, c_size_t, c_uint32, c_uint64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SVGPU_LIB", os.path.join(os.path.dirname(_HERE), "build", "libsvgpu.so"))

SV_CANONICAL = 0
SV_MONTGOMERY = 1

SV_OK, SV_ERR_EMPTY, SV_ERR_LEN, SV_ERR_ARG, SV_ERR_DEVICE, SV_ERR_OOM = range(6)

SV_ENC_HALO2_COMPRESSED = 0
SV_ENC_EVM = 1


class SvError(RuntimeError):
    status = -1


class EmptyError(SvError):
    status = SV_ERR_EMPTY


class LengthError(SvError):
    status = SV_ERR_LEN


class ArgumentError(SvError):
    status = SV_ERR_ARG


class DeviceError(SvError):
    status = SV_ERR_DEVICE


class OutOfMemoryError(SvError):
    status = SV_ERR_OOM


_ERRORS = {c.status: c for c in (EmptyError, LengthError, ArgumentError, DeviceError, OutOfMemoryError)}


class sv_fe(Structure):
    _fields_ = [("l", c_uint64 * 4)]


class sv_g1_affine(Structure):
    _fields_ = [("x", sv_fe), ("y", sv_fe)]


class sv_g1_jacobian(Structure):
    _fields_ = [("x", sv_fe), ("y", sv_fe), ("z", sv_fe)]


class sv_fq2(Structure):
    _fields_ = [("c0", sv_fe), ("c1", sv_fe)]


class sv_g2_affine(Structure):
    _fields_ = [("x", sv_fq2), ("y", sv_fq2)]


class sv_fq12(Structure):
    _fields_ = [("c", sv_fq2 * 6)]


class sv_msm_stats(Structure):
    _fields_ = [
        ("total_ms", c_float), ("digits_ms", c_float), ("sort_ms", c_float), ("accumulate_ms", c_float),
        ("fixup_ms", c_float), ("reduce_ms", c_float), ("host_ms", c_float),
        ("window_bits", c_uint32), ("num_windows", c_uint32), ("accumulate_launch_units", c_uint32),
        ("entries", c_uint64), ("accumulate_span_ms", c_float), ("accumulate_launches", c_uint32),
    ]


# (name, restype, argtypes) -- one row per prototype in include/svgpu.h
PROTOTYPES = [
    ("sv_init", c_int, [c_int]),
    ("sv_device_count", c_int, []),
    ("sv_last_error", c_char_p, []),
    ("sv_version", c_char_p, []),
    ("sv_bn254_g1_msm", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, POINTER(sv_g1_affine)]),
    ("sv_bn254_g1_msm_refs", c_int, [c_void_p, c_size_t, c_int, c_int, POINTER(sv_g1_affine)]),
    ("sv_bn254_g1_msm_device", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p, POINTER(sv_g1_jacobian)]),
    ("sv_bn254_g1_fold", c_int, [c_void_p, c_size_t, POINTER(sv_g1_affine), c_int]),
    ("sv_bn254_kzg_decide", c_int, [POINTER(sv_g2_affine), POINTER(sv_g2_affine), c_void_p, c_void_p, c_size_t,
                                     c_int, c_int, POINTER(c_int32)]),
    ("sv_bn254_kzg_decide_device", c_int, [POINTER(sv_g2_affine), POINTER(sv_g2_affine), c_void_p, c_void_p,
                                            c_size_t, c_int, c_int, c_void_p, POINTER(c_int32), c_void_p, c_void_p]),
    ("sv_bn254_kzg_accumulate", c_int, [c_void_p, c_void_p, c_size_t, POINTER(sv_fe), c_int, c_int,
                                         POINTER(sv_g1_affine), POINTER(sv_g1_affine)]),
    ("sv_bn254_kzg_create_proof", c_int, [c_void_p, c_void_p, c_size_t, c_int, c_int, POINTER(sv_g1_affine),
                                           POINTER(sv_g1_affine), c_void_p, c_void_p]),
    ("sv_bn254_g1_msm_batch", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    ("sv_bn254_g1_msm_batch_device", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_size_t, c_int, c_int,
                                              c_void_p, c_void_p]),
    ("sv_bn254_g1_table_create", c_int, [c_void_p, c_size_t, c_int, c_int, POINTER(c_uint64)]),
    ("sv_bn254_g1_table_destroy", c_int, [c_uint64]),
    ("sv_bn254_g1_msm_batch_table", c_int, [c_uint64, c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_void_p]),
    ("sv_bn254_g1_msm_batch_table_device", c_int, [c_uint64, c_void_p, c_void_p, c_void_p, c_size_t, c_int,
                                                    c_void_p, c_void_p]),
    ("sv_bn254_g1_table_device", c_int, [c_uint64, POINTER(c_int)]),
    ("sv_bn254_g1_msm_batch_indexed_device", c_int, [c_void_p, c_size_t, c_int, c_void_p, c_void_p, c_void_p,
                                                      c_size_t, c_size_t, c_int, c_int, c_void_p, c_void_p]),
    ("sv_bn254_poseidon_permute", c_int, [c_void_p, c_size_t, c_int, c_int]),
    ("sv_bn254_poseidon_permute_device", c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_void_p]),
    ("sv_bn254_poseidon_squeeze", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p]),
    ("sv_bn254_poseidon_squeeze_device", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, c_int, c_int, c_void_p,
                                                  c_int, c_void_p]),
    ("sv_bn254_g1_decode", c_int, [c_void_p, c_size_t, c_int, c_int, c_void_p, POINTER(ctypes.c_int64)]),
    ("sv_bn254_g1_decode_device", c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_void_p, c_void_p,
                                           POINTER(ctypes.c_int64)]),
    ("sv_bn254_kzg_accumulators_from_limbs", c_int, [c_void_p, c_size_t, c_int, c_int, c_int, c_void_p, c_void_p,
                                                      POINTER(ctypes.c_int64)]),
    ("sv_bn254_kzg_decide_eip197", c_int, [c_void_p, c_size_t, c_int, POINTER(c_int32)]),
    ("sv_gen_scalars_device", c_int, [c_void_p, c_size_t, c_uint64, c_uint64, c_int, c_int, c_void_p]),
    ("sv_gen_bases_device", c_int, [c_void_p, c_size_t, c_uint64, c_uint64, c_int, c_int, c_void_p]),
    ("sv_msm_last_stats", c_int, [POINTER(sv_msm_stats)]),
    ("sv_kzg_last_kernel_ms", c_int, [POINTER(c_float)]),
]


def _check_fresh():
    """The library must have been linked from the sources beside it (build/SOURCES.sha256, written
    by the Makefile): a prebuilt .so that travelled with a changed tree raises here.
    SVGPU_ALLOW_STALE=1 skips the check (e.g. an A/B library in another directory)."""
    if os.environ.get("SVGPU_ALLOW_STALE") == "1" or "SVGPU_LIB" in os.environ:
        return
    from ._srchash import source_hash
    stamp = os.path.join(os.path.dirname(LIB_PATH), "SOURCES.sha256")
    want = source_hash()
    have = open(stamp).read().strip() if os.path.exists(stamp) else "(no stamp)"
    if have != want:
        raise ImportError(f"{LIB_PATH} was not built from the current sources (stamp {have[:16]}, sources "
                          f"{want[:16]}): rebuild with `make -C snark-verifier-axiom_amd`")


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libsvgpu.so not found at {LIB_PATH}: build it with `make -C snark-verifier-axiom_amd` "
            "(there is no CPU fallback)")
    _check_fresh()
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def last_error() -> str:
    msg = lib.sv_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "") -> None:
    if rc == SV_OK:
        return
    cls = _ERRORS.get(rc, SvError)
    raise cls(f"{what}: status {rc}: {last_error()}")
