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


# ---- the reference's optimised schedule (OptimizedPoseidonSpec, poseidon.rs:170-328) ---------------
def _mat_mul(a, b, m):
    n = len(a)
    return [[sum(a[i][k] * b[k][j] for k in range(n)) % m for j in range(n)] for i in range(n)]


def _transpose(a):
    return [list(r) for r in zip(*a)]


def _mul_vector(mat, v, m):  # MDSMatrix::mul_vector, poseidon.rs:101-109
    return [sum(mat[i][j] * v[j] for j in range(len(v))) % m for i in range(len(mat))]


def _determinant(mat, m):  # MDSMatrix::determinant, poseidon.rs:139-165 (Gaussian elimination)
    a = [list(r) for r in mat]
    n = len(a)
    res = 1
    for i in range(n):
        piv = i
        while a[piv][i] % m == 0:
            piv += 1
            assert piv < n, "matrix is not invertible"
        if piv != i:
            res = -res
            a[piv], a[i] = a[i], a[piv]
        res = res * a[i][i] % m
        inv = pow(a[i][i], m - 2, m)
        for j in range(i + 1, n):
            f = a[j][i] * inv % m
            for k in range(i + 1, n):
                a[j][k] = (a[j][k] - a[i][k] * f) % m
    return res % m


def _factorise(mat, m):
    """MDSMatrix::factorise (poseidon.rs:167-226): M = M' M'' with M'' sparse ((row, col_hat))."""
    t = len(mat)
    rate = t - 1
    w = [mat[i][0] for i in range(1, t)]
    m_hat = [[mat[i + 1][j + 1] for j in range(rate)] for i in range(rate)]
    det_inv = pow(_determinant(m_hat, m), m - 2, m)
    w_hat = []
    for j in range(rate):  # Cramer's rule: w_hat = m_hat^-1 w
        mj = [list(r) for r in m_hat]
        for i in range(rate):
            mj[i][j] = w[i]
        w_hat.append(_determinant(mj, m) * det_inv % m)
    m_prime = [[1 if i == j else 0 for j in range(t)] for i in range(t)]
    for i in range(rate):
        for j in range(rate):
            m_prime[i + 1][j + 1] = m_hat[i][j]
    m_pp = [[1 if i == j else 0 for j in range(t)] for i in range(t)]
    m_pp[0] = list(mat[0])
    for i in range(rate):
        m_pp[i + 1][0] = w_hat[i]
    row = [m_pp[i][0] for i in range(t)]
    col_hat = m_pp[0][1:]
    return m_prime, (row, col_hat)


@functools.lru_cache(maxsize=None)
def optimized_spec(t: int, r_f: int, r_p: int, modulus: int = FR_MODULUS):
    """OptimizedPoseidonSpec::new (poseidon.rs:230-245): constants (start, partial, end), the dense MDS,
    pre_sparse_mds and the r_p sparse matrices (row, col_hat), from the same Grain constants as spec()."""
    m = modulus
    rc, mds = spec(t, r_f, r_p, m)
    consts = [rc[r * t:(r + 1) * t] for r in range(r_f + r_p)]
    # the inverse MDS (Poseidon128Pow5Gen returns it alongside; Gauss-Jordan here)
    aug = [list(mds[i]) + [1 if i == j else 0 for j in range(t)] for i in range(t)]
    for c in range(t):
        piv = next(r for r in range(c, t) if aug[r][c] % m)
        aug[c], aug[piv] = aug[piv], aug[c]
        inv = pow(aug[c][c], m - 2, m)
        aug[c] = [x * inv % m for x in aug[c]]
        for r in range(t):
            if r != c and aug[r][c]:
                f = aug[r][c]
                aug[r] = [(x - f * y) % m for x, y in zip(aug[r], aug[c])]
    mds_inv = [row[t:] for row in aug]
    half = r_f // 2
    # calculate_optimized_constants, poseidon.rs:247-295
    start = [list(consts[0])] + [_mul_vector(mds_inv, consts[r], m) for r in range(1, half)]
    acc = list(consts[half + r_p])
    partial = [0] * r_p
    for k, c in zip(range(r_p - 1, -1, -1), [consts[r] for r in range(half + r_p - 1, half - 1, -1)]):
        tmp = _mul_vector(mds_inv, acc, m)
        partial[k] = tmp[0]
        tmp[0] = 0
        acc = [(x + y) % m for x, y in zip(tmp, c)]
    start.append(_mul_vector(mds_inv, acc, m))
    end = [_mul_vector(mds_inv, consts[r], m) for r in range(half + r_p + 1, r_f + r_p)]
    # calculate_sparse_matrices, poseidon.rs:297-313
    mds_t = _transpose(mds)
    accm = [list(r) for r in mds_t]
    sparse = []
    for _ in range(r_p):
        m_prime, mpp = _factorise(accm, m)
        accm = _mat_mul(mds_t, m_prime, m)
        sparse.append(mpp)
    sparse.reverse()
    pre_sparse = _transpose(accm)
    return {"start": start, "partial": partial, "end": end, "mds": mds, "pre_sparse": pre_sparse, "sparse": sparse}


def permutation_optimized(state: List[int], t: int, r_f: int, r_p: int, modulus: int = FR_MODULUS) -> List[int]:
    """Poseidon::permutation (poseidon.rs:469-500) without the absorbed inputs and padding: the bare
    HADES map in the reference's optimised schedule; equals permutation() (tests check it)."""
    m = modulus
    sp = optimized_spec(t, r_f, r_p, m)
    st = [(x + c) % m for x, c in zip(state, sp["start"][0])]        # absorb_with_pre_constants
    sbox = lambda v, c: (pow(v, 5, m) + c) % m  # noqa: E731  power5_with_constant
    for cs in sp["start"][1:r_f // 2]:
        st = _mul_vector(sp["mds"], [sbox(v, c) for v, c in zip(st, cs)], m)
    st = _mul_vector(sp["pre_sparse"], [sbox(v, c) for v, c in zip(st, sp["start"][-1])], m)
    for c, (row, col_hat) in zip(sp["partial"], sp["sparse"]):       # sbox_part + apply_sparse_mds
        st[0] = sbox(st[0], c)
        s0 = sum(r * v for r, v in zip(row, st)) % m
        st = [s0] + [(ch * st[0] + v) % m for ch, v in zip(col_hat, st[1:])]
    for cs in sp["end"]:
        st = _mul_vector(sp["mds"], [sbox(v, c) for v, c in zip(st, cs)], m)
    return _mul_vector(sp["mds"], [sbox(v, 0) for v in st], m)


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
