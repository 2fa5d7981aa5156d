"""Poseidon (x^5, BN254 Fr) permutation oracle -- TEST INFRASTRUCTURE ONLY.

Purpose: pin the oracle's Fr arithmetic against the only known-answer vectors the
reference holds, snark-verifier/src/util/hash/poseidon/tests.rs:6-85
(``test_mds`` and ``test_poseidon_against_test_vectors``: HADES vectors
poseidonperm_x5_254_3 and poseidonperm_x5_254_5).

The reference's constants come from the external crate ``poseidon-circuit``
(Spec::constants, Grain-LFSR parameter generation of the Poseidon paper,
eprint 2019/458 Appendix / hadeshash ``generate_parameters_grain.sage``), which is
not vendored.  This module restates that published generator:

* Grain LFSR seeded with (field=1 [2 bits], sbox=0 [4], n [12], t [12], R_F [10],
  R_P [10], thirty 1-bits); 160 warm-up clocks; output bit = second bit of each pair
  whose first bit is 1.
* Round constants: (R_F + R_P) * t draws of n bits, MSB first, rejection-sampled < r.
* MDS: Cauchy matrix 1/(x_i + y_j) from 2t draws of n bits, MSB first, reduced mod r
  (``secure_mds = 0``: the first sampled matrix, as poseidon.rs:230-245 requests).
* Permutation: R_F/2 full rounds, R_P partial rounds (S-box on state[0]), R_F/2 full
  rounds; each round = add constants, S-box x^5, MDS.  This is the unoptimised HADES
  form; the reference's optimised form (poseidon.rs:414-500) computes the same map.

``Sponge`` restates the reference's sponge, Poseidon<F, L, T, RATE> (poseidon.rs:412-500):
state starts (2^64, 0, ..) (State::default, :335-342); ``update`` buffers; ``squeeze``
absorbs RATE-chunks (each added into state[1..], a short chunk padded with a single 1 --
absorb_with_pre_constants, :363-385 -- then permuted), runs one extra permutation of the
padded empty chunk when the buffer length is a multiple of RATE, and returns state[1].
The reference holds no sponge-level vectors: that part is pinned only through the KAT-pinned
permutation plus this line-by-line restatement (parity unpinned at the sponge level).
``transcript_*`` restate PoseidonTranscript<NativeLoader> (system/halo2/transcript/halo2.rs:
198-227): common_scalar = update([s]); common_ec_point = update([x mod r, y mod r])
(fe_to_fe, util/arithmetic.rs:256-258), identity rejected; squeeze_challenge = squeeze().
"""
from __future__ import annotations

import functools
from typing import List, Optional, Sequence

from .bn254 import R as FR_MODULUS


class Grain:
    def __init__(self, n: int, t: int, r_f: int, r_p: int):
        bits: List[int] = []
        for value, width in ((1, 2), (0, 4), (n, 12), (t, 12), (r_f, 10), (r_p, 10)):
            bits.extend(int(c) for c in bin(value)[2:].zfill(width))
        bits.extend([1] * 30)
        assert len(bits) == 80
        self.state = bits
        for _ in range(160):
            self._clock()

    def _clock(self) -> int:
        s = self.state
        b = s[62] ^ s[51] ^ s[38] ^ s[23] ^ s[13] ^ s[0]
        s.pop(0)
        s.append(b)
        return b

    def next_bit(self) -> int:
        while True:
            b1 = self._clock()
            b2 = self._clock()
            if b1:
                return b2

    def next_bits_int(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.next_bit()
        return v


@functools.lru_cache(maxsize=None)
def spec(t: int, r_f: int, r_p: int, modulus: int = FR_MODULUS):
    n = modulus.bit_length()
    g = Grain(n, t, r_f, r_p)
    rc = []
    for _ in range((r_f + r_p) * t):
        while True:
            v = g.next_bits_int(n)
            if v < modulus:
                rc.append(v)
                break
    while True:
        vals = [g.next_bits_int(n) % modulus for _ in range(2 * t)]
        if len(set(vals)) == len(vals):
            break
    xs, ys = vals[:t], vals[t:]
    mds = [[pow((xs[i] + ys[j]) % modulus, modulus - 2, modulus) for j in range(t)] for i in range(t)]
    return rc, mds


def permutation(state: List[int], t: int, r_f: int, r_p: int, modulus: int = FR_MODULUS) -> List[int]:
    rc, mds = spec(t, r_f, r_p, modulus)
    st = [x % modulus for x in state]
    half = r_f // 2
    for rnd in range(r_f + r_p):
        st = [(st[i] + rc[rnd * t + i]) % modulus for i in range(t)]
        if rnd < half or rnd >= half + r_p:
            st = [pow(x, 5, modulus) for x in st]
        else:
            st[0] = pow(st[0], 5, modulus)
        st = [sum(mds[i][j] * st[j] for j in range(t)) % modulus for i in range(t)]
    return st


# widths the reference instantiates: t -> (R_F, R_P)  (tests.rs:39-42, :63-66; sdk halo2.rs:52-55)
PARAMS = {3: (8, 57), 5: (8, 60)}


class Sponge:
    """Poseidon<Fr, Fr, T, RATE> on the NativeLoader (poseidon.rs:412-500)."""

    def __init__(self, t: int = 3, state: Optional[Sequence[int]] = None):
        self.t = t
        self.r_f, self.r_p = PARAMS[t]
        self.rate = t - 1
        self.state = list(state) if state is not None else [1 << 64] + [0] * (t - 1)
        self.buf: List[int] = []

    def clear(self) -> None:
        self.state = [1 << 64] + [0] * (self.t - 1)
        self.buf = []

    def update(self, elements: Sequence[int]) -> None:
        self.buf.extend(int(e) % FR_MODULUS for e in elements)

    def _permutation(self, inputs: Sequence[int]) -> None:
        st = list(self.state)
        for k, x in enumerate(inputs):
            st[1 + k] += x
        if len(inputs) < self.rate:
            st[1 + len(inputs)] += 1
        self.state = permutation(st, self.t, self.r_f, self.r_p)

    def squeeze(self) -> int:
        buf, self.buf = self.buf, []
        for i in range(0, len(buf), self.rate):
            self._permutation(buf[i:i + self.rate])
        if len(buf) % self.rate == 0:
            self._permutation([])
        return self.state[1]


def transcript_common_ec_point(sponge: Sponge, point) -> None:
    if point is None:
        raise ValueError("Invalid elliptic curve point encoding in proof")
    sponge.update([point[0] % FR_MODULUS, point[1] % FR_MODULUS])
