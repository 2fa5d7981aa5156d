"""Host-side mirror of the reference's KZG decider / accumulation, executed on the GPU.

* ``KzgAs.decide`` / ``KzgAs.decide_all`` mirror ``AccumulationDecider for KzgAs`` on
  NativeLoader (snark-verifier/src/pcs/kzg/decider.rs:60-80): pass -> None, failure ->
  ``AssertionFailure("e(lhs, g2)·e(rhs, -s_g2) == O")`` (decider.rs:66-67); an empty list panics
  (``assert!(!accumulators.is_empty())``, decider.rs:74).
* ``KzgAs.create_proof`` / ``KzgAs.verify`` mirror the accumulation MSMs of
  snark-verifier/src/pcs/kzg/accumulation.rs:146-195 / :40-62 without the zk blind:
  lhs = sum r^i lhs_i, rhs = sum r^i rhs_i with r^0 = 1 (snark-verifier/src/loader.rs:71-78).
  ``create_proof(instances, transcript)`` is the reference's own signature: the accumulators' lhs
  and rhs are absorbed through ``transcript.common_ec_point`` and r is squeezed from it
  (accumulation.rs:156-176).  Given a fresh ``PoseidonTranscript`` (what the SDK passes,
  snark-verifier-sdk/src/halo2/aggregation.rs:235-242) the whole call is ONE library call,
  ``sv_bn254_kzg_create_proof`` (host sponge, device MSMs); a used transcript's sponge state goes
  in and comes back out of the same call, and one with buffered input is absorbed and squeezed
  through ``svgpu.poseidon`` first.  An ``int`` in place of the
  transcript is taken as r itself (``sv_bn254_kzg_accumulate``).
"""
from __future__ import annotations

import ctypes
import numbers
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
    def create_proof(instances: Sequence[KzgAccumulator], transcript=None) -> KzgAccumulator:
        """KzgAs::create_proof with the default proving key (no blind), accumulation.rs:146-195.

        ``transcript``: None or a fresh ``PoseidonTranscript`` -> r from the library's transcript
        (one call); a used ``PoseidonTranscript`` -> absorbed / squeezed through it; an integer
        (``numbers.Integral``: int, numpy integers) -> r."""
        if len(instances) == 0:
            raise ReferencePanic("assertion failed: !instances.is_empty()")
        from .poseidon import PoseidonTranscript
        if isinstance(transcript, numbers.Integral):  # int, numpy integers, ...: r itself
            return KzgAs._accumulate(instances, int(transcript))
        if transcript is not None and (not isinstance(transcript, PoseidonTranscript) or transcript.buf.buf
                                       or transcript.buf.t != 3):
            # a transcript with pending input (or another kind): absorb and squeeze through it
            for a in instances:
                transcript.common_ec_point(a.lhs)
                transcript.common_ec_point(a.rhs)
            return KzgAs._accumulate(instances, transcript.squeeze_challenge())
        lhs = enc.bases_array([a.lhs for a in instances])
        rhs = enc.bases_array([a.rhs for a in instances])
        out_l, out_r = _lib.sv_g1_affine(), _lib.sv_g1_affine()
        r = np.zeros(4, dtype=np.uint64)
        state = None
        if transcript is not None:  # continue from the transcript's sponge state, then hand it back
            state = enc.ints_to_limbs([int(v) for v in transcript.buf.state])
        _lib.check(_lib.lib.sv_bn254_kzg_create_proof(lhs.ctypes.data, rhs.ctypes.data, len(instances),
                                                      _lib.SV_CANONICAL, 0, ctypes.byref(out_l), ctypes.byref(out_r),
                                                      None if state is None else state.ctypes.data, r.ctypes.data),
                   "sv_bn254_kzg_create_proof")
        if transcript is not None:
            transcript.buf.state = [enc.limbs_to_int(row) for row in state]
        KzgAs.last_challenge = enc.limbs_to_int(r)
        return KzgAccumulator(enc.g1_from_struct(out_l), enc.g1_from_struct(out_r))

    last_challenge: Optional[int] = None

    @staticmethod
    def _accumulate(instances: Sequence[KzgAccumulator], r: int) -> KzgAccumulator:
        if not 0 <= r < enc.R:
            raise ValueError("r must be a reduced Fr element")
        lhs = enc.bases_array([a.lhs for a in instances])
        rhs = enc.bases_array([a.rhs for a in instances])
        rr = enc.fe_struct(r)
        out_l, out_r = _lib.sv_g1_affine(), _lib.sv_g1_affine()
        _lib.check(_lib.lib.sv_bn254_kzg_accumulate(lhs.ctypes.data, rhs.ctypes.data, len(instances),
                                                    ctypes.byref(rr), _lib.SV_CANONICAL, 0, ctypes.byref(out_l),
                                                    ctypes.byref(out_r)), "sv_bn254_kzg_accumulate")
        KzgAs.last_challenge = r
        return KzgAccumulator(enc.g1_from_struct(out_l), enc.g1_from_struct(out_r))

    @staticmethod
    def verify(instances: Sequence[KzgAccumulator], transcript=None) -> KzgAccumulator:
        """AccumulationScheme::verify (accumulation.rs:40-62): the same transcript and MSMs."""
        return KzgAs.create_proof(instances, transcript)

