"""Host-side mirror of the reference's KZG decider / accumulation, executed on the GPU.

* ``KzgAs.decide`` / ``KzgAs.decide_all`` mirror ``AccumulationDecider for KzgAs`` on
  NativeLoader (snark-verifier/src/pcs/kzg/decider.rs:60-80): pass -> None, failure ->
  ``AssertionFailure("e(lhs, g2)·e(rhs, -s_g2) == O")`` (decider.rs:66-67); an empty list panics
  (``assert!(!accumulators.is_empty())``, decider.rs:74).
* ``KzgAs.create_proof`` / ``KzgAs.verify`` mirror the accumulation MSMs of
  snark-verifier/src/pcs/kzg/accumulation.rs:146-195 / :40-62 without the zk blind:
  lhs = sum r^i lhs_i, rhs = sum r^i rhs_i with r^0 = 1 (snark-verifier/src/loader.rs:71-78).
  The challenge ``r`` is an input: deriving it from the Poseidon transcript is outside the path.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _lib
from . import encoding as enc
from .loader import Point, ReferencePanic

G2Point = Optional[Tuple[Tuple[int, int], Tuple[int, int]]]

DECIDE_MSG = "e(lhs, g2)·e(rhs, -s_g2) == O"


class AssertionFailure(Exception):
    """snark_verifier::Error::AssertionFailure"""


@dataclass(frozen=True)
class KzgDecidingKey:
    """KzgDecidingKey{svk.g, g2, s_g2} (decider.rs:6-30); From<(G1, G2, G2)> (:26-30)."""

    g: Point
    g2: G2Point
    s_g2: G2Point


@dataclass(frozen=True)
class KzgAccumulator:
    """KzgAccumulator{lhs, rhs} (snark-verifier/src/pcs/kzg/accumulator.rs:6-26)."""

    lhs: Point
    rhs: Point


def decide_arrays(dk: KzgDecidingKey, lhs: np.ndarray, rhs: np.ndarray, form: int = _lib.SV_CANONICAL,
                  num_gpus: int = 0) -> int:
    """Batched decider over host arrays (n, 8) u64; returns the first failing index or -1."""
    lhs = np.ascontiguousarray(lhs, dtype=np.uint64)
    rhs = np.ascontiguousarray(rhs, dtype=np.uint64)
    if lhs.shape[0] == 0:
        raise ReferencePanic("assertion failed: !accumulators.is_empty()")
    ff = ctypes.c_int32(-2)
    g2 = enc.g2_struct(dk.g2, form)
    sg2 = enc.g2_struct(dk.s_g2, form)
    _lib.check(_lib.lib.sv_bn254_kzg_decide(ctypes.byref(g2), ctypes.byref(sg2), lhs.ctypes.data, rhs.ctypes.data,
                                            lhs.shape[0], form, num_gpus, ctypes.byref(ff)), "sv_bn254_kzg_decide")
    return ff.value


class KzgAs:
    """KzgAs<Bn256, MOS> on NativeLoader: decider + accumulation (no zk blind)."""

    @staticmethod
    def decide(dk: KzgDecidingKey, acc: KzgAccumulator) -> None:
        KzgAs.decide_all(dk, [acc])

    @staticmethod
    def decide_all(dk: KzgDecidingKey, accumulators: Sequence[KzgAccumulator], num_gpus: int = 0) -> None:
        if len(accumulators) == 0:
            raise ReferencePanic("assertion failed: !accumulators.is_empty()")
        lhs = enc.bases_array([a.lhs for a in accumulators])
        rhs = enc.bases_array([a.rhs for a in accumulators])
        if decide_arrays(dk, lhs, rhs, _lib.SV_CANONICAL, num_gpus) >= 0:
            raise AssertionFailure(DECIDE_MSG)

    @staticmethod
    def first_failure(dk: KzgDecidingKey, accumulators: Sequence[KzgAccumulator], num_gpus: int = 0) -> int:
        lhs = enc.bases_array([a.lhs for a in accumulators])
        rhs = enc.bases_array([a.rhs for a in accumulators])
        return decide_arrays(dk, lhs, rhs, _lib.SV_CANONICAL, num_gpus)

    @staticmethod
    def create_proof(instances: Sequence[KzgAccumulator], r: int) -> KzgAccumulator:
        if len(instances) == 0:
            raise ReferencePanic("assertion failed: !instances.is_empty()")
        if not 0 <= r < enc.R:
            raise ValueError("r must be a reduced Fr element")
        lhs = enc.bases_array([a.lhs for a in instances])
        rhs = enc.bases_array([a.rhs for a in instances])
        rr = enc.fe_struct(r)
        out_l, out_r = _lib.sv_g1_affine(), _lib.sv_g1_affine()
        _lib.check(_lib.lib.sv_bn254_kzg_accumulate(lhs.ctypes.data, rhs.ctypes.data, len(instances),
                                                    ctypes.byref(rr), _lib.SV_CANONICAL, 0, ctypes.byref(out_l),
                                                    ctypes.byref(out_r)), "sv_bn254_kzg_accumulate")
        return KzgAccumulator(enc.g1_from_struct(out_l), enc.g1_from_struct(out_r))

    verify = create_proof  # AccumulationScheme::verify computes the same two MSMs (accumulation.rs:40-62)
