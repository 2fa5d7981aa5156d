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
"""
from __future__ import annotations

from typing import List

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
