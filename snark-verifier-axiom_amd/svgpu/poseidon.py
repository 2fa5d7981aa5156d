"""Poseidon sponge / transcript over BN254 Fr on the GPU.

Mirrors snark-verifier/src/util/hash/poseidon.rs (Poseidon::new / update / squeeze / clear,
:412-467) and the native PoseidonTranscript's Fiat-Shamir calls
(system/halo2/transcript/halo2.rs:198-227).  ``update`` only buffers, exactly like the
reference; every ``squeeze`` is one call of ``sv_bn254_poseidon_squeeze``.  ``squeeze_many``
squeezes many independent sponges (e.g. the transcripts of a batch of snarks) in ONE launch --
one GPU lane per sponge.  No CPU fallback: without libsvgpu / a GPU these raise.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .encoding import R, ints_to_limbs, limbs_to_int

# widths the reference instantiates: t -> (R_F, R_P)  (poseidon/tests.rs:39-42, :63-66;
# snark-verifier-sdk/src/halo2.rs:52-55 uses t = 3 for PoseidonTranscript)
PARAMS = {3: (8, 57), 5: (8, 60)}


def _check_t(t: int) -> None:
    if t not in PARAMS:
        raise _lib.ArgumentError(f"poseidon: unsupported width t = {t} (3 or 5)")


def _fr_array(values: Sequence[int]) -> np.ndarray:
    return ints_to_limbs([int(v) % R for v in values])


def permute(states: Sequence[Sequence[int]], t: int = 3) -> List[List[int]]:
    """HADES permutation of each state (Poseidon::permutation with a full-rate zero input, as the
    reference KATs call it, poseidon/tests.rs:34-85)."""
    _check_t(t)
    if len(states) == 0:
        return []
    for s in states:
        if len(s) != t:
            raise _lib.LengthError(f"poseidon: state of length {len(s)}, expected {t}")
    buf = _fr_array([v for s in states for v in s])
    _lib.check(_lib.lib.sv_bn254_poseidon_permute(buf.ctypes.data, len(states), t, _lib.SV_CANONICAL),
               "sv_bn254_poseidon_permute")
    flat = [limbs_to_int(row) for row in buf]
    return [flat[i * t:(i + 1) * t] for i in range(len(states))]


class Poseidon:
    """Poseidon<Fr, Fr, T, RATE> with the NativeLoader (poseidon.rs:412-467)."""

    def __init__(self, t: int = 3):
        _check_t(t)
        self.t = t
        self.rate = t - 1
        self.state: List[int] = self.default_state(t)
        self.buf: List[int] = []

    @staticmethod
    def default_state(t: int) -> List[int]:
        # State::default (poseidon.rs:335-342): capacity 2^64 + (o - 1), o = 1
        return [1 << 64] + [0] * (t - 1)

    def clear(self) -> None:
        self.state = self.default_state(self.t)
        self.buf = []

    def update(self, elements: Sequence[int]) -> None:
        self.buf.extend(int(e) % R for e in elements)

    def squeeze(self) -> int:
        return squeeze_many([self])[0]


def squeeze_many(sponges: Sequence[Poseidon]) -> List[int]:
    """Poseidon::squeeze on every sponge (all the same width), one kernel launch; returns the
    challenges and leaves each sponge's state updated and buffer empty."""
    if not sponges:
        return []
    t = sponges[0].t
    if any(s.t != t for s in sponges):
        raise _lib.ArgumentError("poseidon: squeeze_many needs sponges of one width")
    n = len(sponges)
    states = _fr_array([v for s in sponges for v in s.state])
    offsets = np.zeros(n + 1, dtype=np.uint64)
    offsets[1:] = np.cumsum([len(s.buf) for s in sponges])
    flat = [e for s in sponges for e in s.buf]
    elements = _fr_array(flat) if flat else np.zeros((1, 4), np.uint64)
    out = np.zeros((n, 4), dtype=np.uint64)
    _lib.check(_lib.lib.sv_bn254_poseidon_squeeze(states.ctypes.data, elements.ctypes.data, offsets.ctypes.data,
                                                  n, t, _lib.SV_CANONICAL, out.ctypes.data),
               "sv_bn254_poseidon_squeeze")
    vals = [limbs_to_int(row) for row in states]
    for i, s in enumerate(sponges):
        s.state = vals[i * t:(i + 1) * t]
        s.buf = []
    return [limbs_to_int(row) for row in out]


class PoseidonTranscript:
    """Fiat-Shamir side of PoseidonTranscript<NativeLoader> (halo2.rs:198-227), t = 3 (the SDK's)."""

    def __init__(self, t: int = 3):
        self.buf = Poseidon(t)

    def common_scalar(self, scalar: int) -> None:
        self.buf.update([scalar])

    def common_ec_point(self, point: Optional[tuple]) -> None:
        # coordinates() is None for the identity -> Error::Transcript (halo2.rs:215-223)
        if point is None:
            raise ValueError("Invalid elliptic curve point encoding in proof")
        # fe_to_fe: Fq -> Fr by reduction mod r (util/arithmetic.rs:256-258)
        self.buf.update([point[0] % R, point[1] % R])

    def squeeze_challenge(self) -> int:
        return self.buf.squeeze()
