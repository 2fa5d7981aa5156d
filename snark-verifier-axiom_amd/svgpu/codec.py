"""Codecs on either side of the path, decoded on the GPU.

* ``read_ec_points(data, encoding)`` -- batched ``read_ec_point`` of the two transcripts:
  halo2curves' 32-byte compressed G1 (PoseidonTranscript, system/halo2/transcript/halo2.rs:247-260)
  or 64-byte big-endian x || y (EvmTranscript, system/halo2/transcript/evm.rs:223-242).
  An invalid encoding raises :class:`TranscriptError` with the reference's message.
* ``LimbsEncoding(LIMBS, BITS).from_repr(limbs)`` -- pcs/kzg/accumulator.rs:57-77 (the SDK's
  LIMBS = 3, BITS = 88); ``from_repr_many`` decodes a batch in one launch.
* ``eip197_input(dk, acc)`` -- the ecPairing input the EVM decider builds (pcs/kzg/decider.rs:107-127);
  ``decide_eip197(records)`` decides a batch of such records on the GPU.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence

import numpy as np

from . import _lib
from . import encoding as enc
from .kzg import KzgAccumulator
from .loader import ReferencePanic

POINT_MSG = "Invalid elliptic curve point encoding in proof"
P = enc.P


class TranscriptError(ValueError):
    """Error::Transcript(io::ErrorKind::Other, "Invalid elliptic curve point encoding in proof")."""

    def __init__(self, index: int):
        super().__init__(POINT_MSG)
        self.index = index


def read_ec_points(data: bytes, encoding: int = _lib.SV_ENC_HALO2_COMPRESSED) -> list:
    rec = 64 if encoding == _lib.SV_ENC_EVM else 32
    if len(data) % rec:
        raise _lib.LengthError(f"encoded points must be a multiple of {rec} bytes")
    n = len(data) // rec
    if n == 0:
        return []
    buf = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros((n, 8), dtype=np.uint64)
    bad = ctypes.c_int64(-1)
    rc = _lib.lib.sv_bn254_g1_decode(buf.ctypes.data, n, encoding, _lib.SV_CANONICAL, out.ctypes.data,
                                     ctypes.byref(bad))
    if rc == _lib.SV_ERR_ARG and bad.value >= 0:
        raise TranscriptError(bad.value)
    _lib.check(rc, "sv_bn254_g1_decode")
    return [enc.g1_from_limbs(r) for r in out]


def _g2_words(q) -> bytes:
    (x0, x1), (y0, y1) = q
    return b"".join(int(v).to_bytes(32, "big") for v in (x1, x0, y1, y0))


def _g1_evm(pt) -> bytes:
    if pt is None:
        return b"\0" * 64
    return int(pt[0]).to_bytes(32, "big") + int(pt[1]).to_bytes(32, "big")


def eip197_input(dk, acc: KzgAccumulator) -> bytes:
    """lhs, g2, rhs, -s_g2 (0x180 bytes) as pcs/kzg/decider.rs:107-127 + loader/evm/loader.rs:338-382."""
    (x0, x1), (y0, y1) = dk.s_g2
    minus_s_g2 = ((x0, x1), ((P - y0) % P, (P - y1) % P))
    return _g1_evm(acc.lhs) + _g2_words(dk.g2) + _g1_evm(acc.rhs) + _g2_words(minus_s_g2)


def decide_eip197(records: bytes) -> int:
    """First failing check of a batch of 0x180-byte EIP-197 records (-1: all pass)."""
    if len(records) % 0x180:
        raise _lib.LengthError("EIP-197 input must be 0x180 bytes per pairing check")
    n = len(records) // 0x180
    if n == 0:
        raise ReferencePanic("assertion failed: !accumulators.is_empty()")
    buf = np.frombuffer(bytes(records), dtype=np.uint8)
    ff = ctypes.c_int32(-2)
    _lib.check(_lib.lib.sv_bn254_kzg_decide_eip197(buf.ctypes.data, n, 0, ctypes.byref(ff)),
               "sv_bn254_kzg_decide_eip197")
    return ff.value


class LimbsEncoding:
    """LimbsEncoding<LIMBS, BITS> as an AccumulatorEncoding on the NativeLoader."""

    def __init__(self, limbs: int = 3, bits: int = 88):
        self.limbs = limbs
        self.bits = bits

    def from_repr(self, limbs: Sequence[int]) -> KzgAccumulator:
        return self.from_repr_many([limbs])[0]

    def from_repr_many(self, batch: Sequence[Sequence[int]]) -> List[KzgAccumulator]:
        for ls in batch:
            if len(ls) != 4 * self.limbs:
                raise ReferencePanic("assertion failed: limbs.len() == 4 * LIMBS")
        n = len(batch)
        if n == 0:
            return []
        arr = enc.scalars_array([int(v) for ls in batch for v in ls])
        lhs = np.zeros((n, 8), dtype=np.uint64)
        rhs = np.zeros((n, 8), dtype=np.uint64)
        bad = ctypes.c_int64(-1)
        rc = _lib.lib.sv_bn254_kzg_accumulators_from_limbs(arr.ctypes.data, n, self.limbs, self.bits,
                                                          _lib.SV_CANONICAL, lhs.ctypes.data, rhs.ctypes.data,
                                                          ctypes.byref(bad))
        if rc == _lib.SV_ERR_ARG and bad.value >= 0:
            # fe_from_big(..) / C::from_xy(..) unwrap on a bad value (accumulator.rs:60-73)
            raise ReferencePanic(f"called `Option::unwrap()` on a `None` value (accumulator {bad.value})")
        _lib.check(rc, "sv_bn254_kzg_accumulators_from_limbs")
        return [KzgAccumulator(enc.g1_from_limbs(a), enc.g1_from_limbs(b)) for a, b in zip(lhs, rhs)]
