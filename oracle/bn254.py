"""BN254 CPU oracle in pure Python -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module, and only as a checker.  The product path (``libsvgpu.so``
and the ``svgpu`` package) never calls it.

What it restates (reference = yuliakot/snark-verifier-axiom, read as text):

* ``native_msm``  -- ``NativeLoader::multi_scalar_multiplication``
  (snark-verifier/src/loader/native.rs:61-71): sum_i base_i * scalar_i, then
  ``to_affine``; panics on empty input (:69).
* ``pippenger_msm`` -- ``util::msm::multi_scalar_multiplication_serial``
  (snark-verifier/src/util/msm.rs:238-283) incl. the ``Bucket`` enum
  (msm.rs:207-236), the window heuristic c = ceil(ln n) + 2 (:247) and the
  byte-window extraction (:250-260).  ``pippenger_msm_parallel`` restates the
  rayon chunking of msm.rs:287-316.
* ``decide`` / ``decide_all`` -- ``AccumulationDecider for KzgAs`` on
  NativeLoader (snark-verifier/src/pcs/kzg/decider.rs:60-80):
  e(lhs, g2) * e(rhs, -s_g2) == 1.
* ``accumulate`` -- ``KzgAs::create_proof`` without zk blind
  (snark-verifier/src/pcs/kzg/accumulation.rs:146-195) with powers of r
  starting at 1 (snark-verifier/src/loader.rs:71-78).
* ``fe_to_limbs``/``fe_from_limbs`` -- snark-verifier/src/util/arithmetic.rs:262-290;
  ``accumulator_from_limbs`` -- LimbsEncoding::from_repr (pcs/kzg/accumulator.rs:57-77).
* point codecs: ``g1_decompress`` (halo2curves compressed, read by transcript/halo2.rs:247-260),
  ``g1_evm_decode`` (transcript/evm.rs:223-242), ``eip197_input`` (pcs/kzg/decider.rs:107-127).

The field/curve/pairing arithmetic itself lives in the un-vendored dependency
halo2curves 0.3.1 (axiom-crypto/halo2 @ 98bc83b, Cargo.lock:1820-1823), which
is absent here.  It is restated from the public BN254 (alt_bn128) definition:
p, r, b = 3, G1 = (1, 2), Fq2 = Fq[u]/(u^2+1), xi = 9+u, Fq6 = Fq2[v]/(v^3-xi),
Fq12 = Fq6[w]/(w^2-v), D-type sextic twist y^2 = x^3 + 3/xi, optimal-ate loop
on 6x+2.  halo2curves keeps Fq/Fr as 4 x u64 little-endian Montgomery limbs
with R = 2^256; identity affine = (0, 0).

PARITY STATUS.  The reference ships no BN254 MSM / pairing vectors
(SURVEY.md section 8c), so MSM and pairing outputs are *parity unpinned* against
the reference itself.  This oracle is pinned instead by (1) the reference's
only known-answer tests -- the Poseidon KATs in
snark-verifier/src/util/hash/poseidon/tests.rs:6-85, which pin Fr arithmetic
(see ``oracle/poseidon.py``); (2) algebraic identities (group law, r*P = O,
bilinearity, non-degeneracy); (3) two independent pairing formulations
(sparse-line tower Miller loop vs. a generic Fq12 polynomial-basis Miller loop
with a direct (p^12-1)/r exponentiation) which must agree on Gt values.
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional, Sequence, Tuple

# ----------------------------------------------------------------------------
# Constants
# ----------------------------------------------------------------------------
P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
U = 4965661367192848881  # BN parameter x (positive for BN254)
B = 3
MONT_R_BITS = 256
RP = (1 << 256) % P  # Montgomery R mod p
RR = (1 << 256) % R  # Montgomery R mod r

assert P == 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1
assert R == 36 * U**4 + 36 * U**3 + 18 * U**2 + 6 * U + 1


def inv(a: int, m: int = P) -> int:
    a %= m
    if a == 0:
        raise ZeroDivisionError("inverse of zero")
    return pow(a, m - 2, m)


def sqrt_fp(a: int) -> Optional[int]:
    """p = 3 mod 4 square root; None for a non-residue."""
    a %= P
    y = pow(a, (P + 1) // 4, P)
    return y if y * y % P == a else None


# ----------------------------------------------------------------------------
# Fq2 = Fq[u]/(u^2 + 1), elements as tuples (c0, c1)
# ----------------------------------------------------------------------------
F2_ZERO = (0, 0)
F2_ONE = (1, 0)
XI = (9, 1)


def f2_add(a, b):
    return ((a[0] + b[0]) % P, (a[1] + b[1]) % P)


def f2_sub(a, b):
    return ((a[0] - b[0]) % P, (a[1] - b[1]) % P)


def f2_neg(a):
    return ((-a[0]) % P, (-a[1]) % P)


def f2_mul(a, b):
    t0 = a[0] * b[0]
    t1 = a[1] * b[1]
    return ((t0 - t1) % P, ((a[0] + a[1]) * (b[0] + b[1]) - t0 - t1) % P)


def f2_sqr(a):
    return f2_mul(a, a)


def f2_mul_fp(a, s):
    return (a[0] * s % P, a[1] * s % P)


def f2_conj(a):
    return (a[0], (-a[1]) % P)


def f2_inv(a):
    t = inv(a[0] * a[0] + a[1] * a[1])
    return (a[0] * t % P, (-a[1]) * t % P)


def f2_mul_xi(a):
    # (a0 + a1 u)(9 + u) = (9 a0 - a1) + (a0 + 9 a1) u
    return ((9 * a[0] - a[1]) % P, (a[0] + 9 * a[1]) % P)


def f2_pow(a, e):
    r = F2_ONE
    while e:
        if e & 1:
            r = f2_mul(r, a)
        a = f2_sqr(a)
        e >>= 1
    return r


# ----------------------------------------------------------------------------
# Fq6 = Fq2[v]/(v^3 - xi), elements (c0, c1, c2)
# ----------------------------------------------------------------------------
F6_ZERO = (F2_ZERO, F2_ZERO, F2_ZERO)
F6_ONE = (F2_ONE, F2_ZERO, F2_ZERO)


def f6_add(a, b):
    return (f2_add(a[0], b[0]), f2_add(a[1], b[1]), f2_add(a[2], b[2]))


def f6_sub(a, b):
    return (f2_sub(a[0], b[0]), f2_sub(a[1], b[1]), f2_sub(a[2], b[2]))


def f6_neg(a):
    return (f2_neg(a[0]), f2_neg(a[1]), f2_neg(a[2]))


def f6_mul(a, b):
    t0 = f2_mul(a[0], b[0])
    t1 = f2_mul(a[1], b[1])
    t2 = f2_mul(a[2], b[2])
    c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a[1], a[2]), f2_add(b[1], b[2])), t1), t2)))
    c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a[0], a[1]), f2_add(b[0], b[1])), t0), t1), f2_mul_xi(t2))
    c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a[0], a[2]), f2_add(b[0], b[2])), t0), t2), t1)
    return (c0, c1, c2)


def f6_mul_by_v(a):
    return (f2_mul_xi(a[2]), a[0], a[1])


def f6_mul_f2(a, s):
    return (f2_mul(a[0], s), f2_mul(a[1], s), f2_mul(a[2], s))


def f6_inv(a):
    a0, a1, a2 = a
    t0 = f2_sub(f2_sqr(a0), f2_mul_xi(f2_mul(a1, a2)))
    t1 = f2_sub(f2_mul_xi(f2_sqr(a2)), f2_mul(a0, a1))
    t2 = f2_sub(f2_sqr(a1), f2_mul(a0, a2))
    d = f2_add(f2_mul(a0, t0), f2_mul_xi(f2_add(f2_mul(a2, t1), f2_mul(a1, t2))))
    di = f2_inv(d)
    return (f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di))


# ----------------------------------------------------------------------------
# Fq12 = Fq6[w]/(w^2 - v), elements (c0, c1)
# basis order used by the C-ABI's Gt layout: c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2
# ----------------------------------------------------------------------------
F12_ONE = (F6_ONE, F6_ZERO)


def f12_mul(a, b):
    t0 = f6_mul(a[0], b[0])
    t1 = f6_mul(a[1], b[1])
    c0 = f6_add(t0, f6_mul_by_v(t1))
    c1 = f6_sub(f6_sub(f6_mul(f6_add(a[0], a[1]), f6_add(b[0], b[1])), t0), t1)
    return (c0, c1)


def f12_sqr(a):
    return f12_mul(a, a)


def f12_conj(a):
    return (a[0], f6_neg(a[1]))


def f12_inv(a):
    t = f6_sub(f6_mul(a[0], a[0]), f6_mul_by_v(f6_mul(a[1], a[1])))
    ti = f6_inv(t)
    return (f6_mul(a[0], ti), f6_neg(f6_mul(a[1], ti)))


def f12_pow(a, e):
    r = F12_ONE
    while e:
        if e & 1:
            r = f12_mul(r, a)
        a = f12_sqr(a)
        e >>= 1
    return r


# Frobenius: an Fq12 element is sum_k g_k w^k with g_k in Fq2 where
#   k=0 -> c0.c0, k=2 -> c0.c1, k=4 -> c0.c2, k=1 -> c1.c0, k=3 -> c1.c1, k=5 -> c1.c2.
# (g w^k)^p = conj(g) * w^k * xi^(k (p-1)/6).
FROB_GAMMA = [f2_pow(XI, k * (P - 1) // 6) for k in range(6)]


def f12_frob(a):
    c0, c1 = a
    g = FROB_GAMMA
    return (
        (f2_conj(c0[0]), f2_mul(f2_conj(c0[1]), g[2]), f2_mul(f2_conj(c0[2]), g[4])),
        (f2_mul(f2_conj(c1[0]), g[1]), f2_mul(f2_conj(c1[1]), g[3]), f2_mul(f2_conj(c1[2]), g[5])),
    )


def f12_frob_n(a, n):
    for _ in range(n):
        a = f12_frob(a)
    return a


def f12_is_one(a):
    return a == F12_ONE


def f12_to_list(a) -> List[int]:
    """Flatten to 12 canonical Fq ints in the C-ABI Gt order."""
    out = []
    for c6 in a:
        for c2 in c6:
            out.extend([c2[0] % P, c2[1] % P])
    return out


# ----------------------------------------------------------------------------
# G1: y^2 = x^3 + 3 over Fq. Affine None = identity; Jacobian (X, Y, Z) with Z=0 identity.
# ----------------------------------------------------------------------------
G1_GEN = (1, 2)


def g1_on_curve(pt) -> bool:
    if pt is None:
        return True
    x, y = pt
    return (y * y - x * x * x - B) % P == 0


def g1_neg(pt):
    if pt is None:
        return None
    return (pt[0], (-pt[1]) % P)


def jac_from_affine(pt):
    if pt is None:
        return (1, 1, 0)
    return (pt[0], pt[1], 1)


def jac_to_affine(p):
    X, Y, Z = p
    if Z % P == 0:
        return None
    zi = inv(Z)
    zi2 = zi * zi % P
    return (X * zi2 % P, Y * zi2 * zi % P)


def jac_double(p):
    X, Y, Z = p
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    A = X * X % P
    Bq = Y * Y % P
    C = Bq * Bq % P
    D = 2 * ((X + Bq) ** 2 - A - C) % P
    E = 3 * A % P
    F = E * E % P
    X3 = (F - 2 * D) % P
    Y3 = (E * (D - X3) - 8 * C) % P
    Z3 = 2 * Y * Z % P
    return (X3, Y3, Z3)


def jac_add(p, q):
    X1, Y1, Z1 = p
    X2, Y2, Z2 = q
    if Z1 == 0:
        return q
    if Z2 == 0:
        return p
    Z1Z1 = Z1 * Z1 % P
    Z2Z2 = Z2 * Z2 % P
    U1 = X1 * Z2Z2 % P
    U2 = X2 * Z1Z1 % P
    S1 = Y1 * Z2 * Z2Z2 % P
    S2 = Y2 * Z1 * Z1Z1 % P
    if U1 == U2:
        if S1 == S2:
            return jac_double(p)
        return (1, 1, 0)
    H = (U2 - U1) % P
    I = (2 * H) ** 2 % P
    J = H * I % P
    r = 2 * (S2 - S1) % P
    V = U1 * I % P
    X3 = (r * r - J - 2 * V) % P
    Y3 = (r * (V - X3) - 2 * S1 * J) % P
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % P
    return (X3, Y3, Z3)


def jac_add_affine(p, q):
    return jac_add(p, jac_from_affine(q))


def jac_neg(p):
    return (p[0], (-p[1]) % P, p[2])


def jac_mul(p, k: int):
    """Double-and-add, MSB first (the group law does not depend on the chain)."""
    acc = (1, 1, 0)
    for bit in bin(k)[2:] if k > 0 else "":
        acc = jac_double(acc)
        if bit == "1":
            acc = jac_add(acc, p)
    return acc


def g1_add(a, b):
    return jac_to_affine(jac_add(jac_from_affine(a), jac_from_affine(b)))


def g1_mul(pt, k: int):
    return jac_to_affine(jac_mul(jac_from_affine(pt), k % R))


def g1_eq(a, b) -> bool:
    return a == b


# ----------------------------------------------------------------------------
# G2 on the D-type twist E': y^2 = x^3 + 3/xi over Fq2
# ----------------------------------------------------------------------------
B2 = f2_mul_fp(f2_inv(XI), 3)
G2_GEN = (
    (10857046999023057135944570762232829481370756359578518086990519993285655852781,
     11559732032986387107991004021392285783925812861821192530917403151452391805634),
    (8495653923123431417604973247489272438418190587263600148770280649306958101930,
     4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def g2_on_curve(q) -> bool:
    if q is None:
        return True
    x, y = q
    return f2_sub(f2_sqr(y), f2_add(f2_mul(f2_sqr(x), x), B2)) == F2_ZERO


def g2_neg(q):
    if q is None:
        return None
    return (q[0], f2_neg(q[1]))


def g2_add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    (x1, y1), (x2, y2) = a, b
    if x1 == x2:
        if y1 == y2:
            if y1 == F2_ZERO:
                return None
            lam = f2_mul(f2_mul_fp(f2_sqr(x1), 3), f2_inv(f2_mul_fp(y1, 2)))
        else:
            return None
    else:
        lam = f2_mul(f2_sub(y2, y1), f2_inv(f2_sub(x2, x1)))
    x3 = f2_sub(f2_sub(f2_sqr(lam), x1), x2)
    y3 = f2_sub(f2_mul(lam, f2_sub(x1, x3)), y1)
    return (x3, y3)


def g2_mul(q, k: int):
    acc = None
    k %= R
    for bit in bin(k)[2:] if k > 0 else "":
        acc = g2_add(acc, acc)
        if bit == "1":
            acc = g2_add(acc, q)
    return acc


# Frobenius endomorphism on the twist (untwist-Frobenius-twist), used for Q1 = pi(Q), Q2 = -pi^2(Q)
TWIST_FROB_X = f2_pow(XI, (P - 1) // 3)
TWIST_FROB_Y = f2_pow(XI, (P - 1) // 2)


def g2_frob(q):
    x, y = q
    return (f2_mul(f2_conj(x), TWIST_FROB_X), f2_mul(f2_conj(y), TWIST_FROB_Y))


# ----------------------------------------------------------------------------
# Optimal-ate pairing, formulation A: projective Miller loop with D-type sparse
# lines (the formulation the C++ oracle and the HIP kernels implement).
# ----------------------------------------------------------------------------
def naf(k: int) -> List[int]:
    """Non-adjacent form, least-significant digit first."""
    out = []
    while k > 0:
        if k & 1:
            d = 2 - (k % 4)
            k -= d
        else:
            d = 0
        out.append(d)
        k >>= 1
    return out


ATE_LOOP_NAF = naf(6 * U + 2)  # 65 digits, LSB first
TWO_INV = inv(2)


def _doubling_step(T):
    """T = (X, Y, Z) homogeneous projective over Fq2; returns (T', coeffs)."""
    X, Y, Z = T
    a = f2_mul_fp(f2_mul(X, Y), TWO_INV)
    b = f2_sqr(Y)
    c = f2_sqr(Z)
    e = f2_mul(B2, f2_mul_fp(c, 3))
    f = f2_mul_fp(e, 3)
    g = f2_mul_fp(f2_add(b, f), TWO_INV)
    h = f2_sub(f2_sqr(f2_add(Y, Z)), f2_add(b, c))
    i = f2_sub(e, b)
    j = f2_sqr(X)
    e2 = f2_sqr(e)
    X3 = f2_mul(a, f2_sub(b, f))
    Y3 = f2_sub(f2_sqr(g), f2_mul_fp(e2, 3))
    Z3 = f2_mul(b, h)
    return (X3, Y3, Z3), (f2_neg(h), f2_mul_fp(j, 3), i)


def _addition_step(T, Q):
    X, Y, Z = T
    qx, qy = Q
    theta = f2_sub(Y, f2_mul(qy, Z))
    lam = f2_sub(X, f2_mul(qx, Z))
    c = f2_sqr(theta)
    d = f2_sqr(lam)
    e = f2_mul(lam, d)
    f = f2_mul(Z, c)
    g = f2_mul(X, d)
    h = f2_sub(f2_add(e, f), f2_mul_fp(g, 2))
    X3 = f2_mul(lam, h)
    Y3 = f2_sub(f2_mul(theta, f2_sub(g, h)), f2_mul(e, Y))
    Z3 = f2_mul(Z, e)
    j = f2_sub(f2_mul(theta, qx), f2_mul(lam, qy))
    return (X3, Y3, Z3), (lam, f2_neg(theta), j)


def g2_prepare(Q) -> List[Tuple]:
    """Line coefficients (c0, c1, c2) in Fq2 for every Miller-loop step (88 for BN254)."""
    T = (Q[0], Q[1], F2_ONE)
    negQ = g2_neg(Q)
    coeffs = []
    for d in reversed(ATE_LOOP_NAF[:-1]):
        T, c = _doubling_step(T)
        coeffs.append(c)
        if d == 1:
            T, c = _addition_step(T, Q)
            coeffs.append(c)
        elif d == -1:
            T, c = _addition_step(T, negQ)
            coeffs.append(c)
    Q1 = g2_frob(Q)
    Q2 = g2_neg(g2_frob(Q1))
    T, c = _addition_step(T, Q1)
    coeffs.append(c)
    T, c = _addition_step(T, Q2)
    coeffs.append(c)
    return coeffs


def f12_mul_by_034(f, c0, c3, c4):
    """f * (c0 + c3 w + c4 v w): sparse line (positions 0, 3, 4 of the 1,v,v^2,w,vw,v^2w basis)."""
    line = ((c0, F2_ZERO, F2_ZERO), (c3, c4, F2_ZERO))
    return f12_mul(f, line)


def _ell(f, coeff, p):
    c0 = f2_mul_fp(coeff[0], p[1])
    c1 = f2_mul_fp(coeff[1], p[0])
    return f12_mul_by_034(f, c0, c1, coeff[2])


def multi_miller_loop(terms: Sequence[Tuple]) -> Tuple:
    """terms: [(G1 affine or None, prepared coeff list or None)]; identity terms are skipped."""
    pairs = [(p, c) for (p, c) in terms if p is not None and c is not None]
    f = F12_ONE
    idx = 0
    n = len(ATE_LOOP_NAF)
    for i in range(n - 1, 0, -1):
        if i != n - 1:
            f = f12_sqr(f)
        for p, c in pairs:
            f = _ell(f, c[idx], p)
        idx += 1
        d = ATE_LOOP_NAF[i - 1]
        if d != 0:
            for p, c in pairs:
                f = _ell(f, c[idx], p)
            idx += 1
    for p, c in pairs:
        f = _ell(f, c[idx], p)
    idx += 1
    for p, c in pairs:
        f = _ell(f, c[idx], p)
    idx += 1
    return f


FINAL_EXP_HARD = (P**4 - P**2 + 1) // R
assert (P**4 - P**2 + 1) % R == 0


def final_exponentiation(f):
    """Exact f^((p^12-1)/r): easy part (p^6-1)(p^2+1), then the hard part
    (p^4-p^2+1)/r through its p-adic digits (lam0 + lam1 p + lam2 p^2 + p^3) with
    lam2 = 6x^2+1, lam1 = -36x^3-18x^2-12x+1, lam0 = -36x^3-30x^2-18x-2
    (exact, not a multiple -- checked against the direct power in tests)."""
    f = f12_mul(f12_conj(f), f12_inv(f))
    f = f12_mul(f12_frob_n(f, 2), f)
    return final_exp_hard_chain(f)


def final_exp_hard_chain(f):
    fx = f12_pow(f, U)
    fx2 = f12_pow(fx, U)
    fx3 = f12_pow(fx2, U)
    # unitary: inverse == conjugate
    l2 = f12_mul(f12_pow(fx2, 6), f)
    l1 = f12_mul(f12_conj(f12_mul(f12_mul(f12_pow(fx3, 36), f12_pow(fx2, 18)), f12_pow(fx, 12))), f)
    l0 = f12_conj(f12_mul(f12_mul(f12_mul(f12_pow(fx3, 36), f12_pow(fx2, 30)), f12_pow(fx, 18)), f12_sqr(f)))
    return f12_mul(f12_mul(f12_mul(l0, f12_frob(l1)), f12_frob_n(l2, 2)), f12_frob_n(f, 3))


def pairing(p, q):
    """e(P, Q) with P in G1 (affine), Q in G2 (affine twist coords)."""
    if p is None or q is None:
        return F12_ONE
    return final_exponentiation(multi_miller_loop([(p, g2_prepare(q))]))


# ----------------------------------------------------------------------------
# Formulation B (independent cross-check): generic Fq12 = Fq[w]/(w^12 - 18 w^6 + 82),
# untwisted Q, affine lines, direct exponentiation by (p^12-1)/r.
# ----------------------------------------------------------------------------
_MODC = [82, 0, 0, 0, 0, 0, -18, 0, 0, 0, 0, 0]  # w^12 = 18 w^6 - 82


def _p12_mul(a, b):
    prod = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                prod[i + j] += ai * bj
    for k in range(22, 11, -1):
        c = prod[k]
        if c:
            prod[k] = 0
            prod[k - 6] += 18 * c
            prod[k - 12] -= 82 * c
    return [x % P for x in prod[:12]]


def _p12_one():
    return [1] + [0] * 11


def _p12_inv(a):
    # extended Euclid over Fq[w]
    lm, hm = [1] + [0] * 12, [0] * 13
    low, high = list(a) + [0], [82, 0, 0, 0, 0, 0, (-18) % P, 0, 0, 0, 0, 0, 1]

    def deg(p):
        d = len(p) - 1
        while d and p[d] % P == 0:
            d -= 1
        return d

    while deg(low):
        r = [0] * 13
        # poly division high / low
        hi = list(high)
        dl = deg(low)
        dh = deg(hi)
        inv_lead = inv(low[dl])
        while dh >= dl and any(x % P for x in hi):
            c = hi[dh] * inv_lead % P
            r[dh - dl] = c
            for i in range(dl + 1):
                hi[dh - dl + i] = (hi[dh - dl + i] - c * low[i]) % P
            if dh == 0:
                break
            dh = deg(hi)
            if hi[dh] % P == 0:
                break
        nm = list(hm)
        new = list(high)
        for i in range(13):
            for j in range(13 - i):
                nm[i + j] -= lm[i] * r[j]
                new[i + j] -= low[i] * r[j]
        nm = [x % P for x in nm]
        new = [x % P for x in new]
        lm, low, hm, high = nm, new, lm, low
    c = inv(low[0])
    return [x * c % P for x in lm[:12]]


def _p12_pow(a, e):
    r = _p12_one()
    while e:
        if e & 1:
            r = _p12_mul(r, a)
        a = _p12_mul(a, a)
        e >>= 1
    return r


def _fq2_to_p12(a):
    # u = w^6 - 9
    out = [0] * 12
    out[0] = (a[0] - 9 * a[1]) % P
    out[6] = a[1] % P
    return out


def tower_to_poly(f) -> List[int]:
    """Map a tower Fq12 element to the w-polynomial basis (w^2 = v, w^6 = xi)."""
    out = [0] * 12
    pos = {(0, 0): 0, (0, 1): 2, (0, 2): 4, (1, 0): 1, (1, 1): 3, (1, 2): 5}
    for i in range(2):
        for j in range(3):
            c = _fq2_to_p12(f[i][j])
            k = pos[(i, j)]
            for t in range(12):
                if c[t]:
                    idx = t + k
                    if idx >= 12:
                        # multiply by w^12 = 18 w^6 - 82
                        out[idx - 6] += 18 * c[t]
                        out[idx - 12] -= 82 * c[t]
                    else:
                        out[idx] += c[t]
    return [x % P for x in out]


def pairing_generic(p, q) -> List[int]:
    """py_ecc-style optimal ate on the untwisted curve over Fq12 (independent code path)."""
    if p is None or q is None:
        return _p12_one()
    w2 = [0, 0, 1] + [0] * 9
    w3 = [0, 0, 0, 1] + [0] * 8
    # untwist (x', y') -> (x' w^2, y' w^3)
    Qx = _p12_mul(_fq2_to_p12(q[0]), w2)
    Qy = _p12_mul(_fq2_to_p12(q[1]), w3)
    Px = [p[0]] + [0] * 11
    Py = [p[1]] + [0] * 11

    def sub(a, b):
        return [(x - y) % P for x, y in zip(a, b)]

    def add(a, b):
        return [(x + y) % P for x, y in zip(a, b)]

    def scal(a, s):
        return [x * s % P for x in a]

    def pt_add(A, Bp):
        if A is None:
            return Bp
        if Bp is None:
            return A
        (x1, y1), (x2, y2) = A, Bp
        if x1 == x2:
            if y1 == y2:
                lam = _p12_mul(scal(_p12_mul(x1, x1), 3), _p12_inv(scal(y1, 2)))
            else:
                return None
        else:
            lam = _p12_mul(sub(y2, y1), _p12_inv(sub(x2, x1)))
        x3 = sub(sub(_p12_mul(lam, lam), x1), x2)
        y3 = sub(_p12_mul(lam, sub(x1, x3)), y1)
        return (x3, y3)

    def line(A, Bp):
        (x1, y1), (x2, y2) = A, Bp
        if x1 != x2:
            lam = _p12_mul(sub(y2, y1), _p12_inv(sub(x2, x1)))
            return sub(_p12_mul(lam, sub(Px, x1)), sub(Py, y1))
        if y1 == y2:
            lam = _p12_mul(scal(_p12_mul(x1, x1), 3), _p12_inv(scal(y1, 2)))
            return sub(_p12_mul(lam, sub(Px, x1)), sub(Py, y1))
        return sub(Px, x1)

    def frob_pt(A):
        return (_p12_pow(A[0], P), _p12_pow(A[1], P))

    Q = (Qx, Qy)
    T = Q
    f = _p12_one()
    loop = 6 * U + 2
    for i in range(loop.bit_length() - 2, -1, -1):
        f = _p12_mul(_p12_mul(f, f), line(T, T))
        T = pt_add(T, T)
        if (loop >> i) & 1:
            f = _p12_mul(f, line(T, Q))
            T = pt_add(T, Q)
    Q1 = frob_pt(Q)
    nQ2 = frob_pt(Q1)
    nQ2 = (nQ2[0], [(-x) % P for x in nQ2[1]])
    f = _p12_mul(f, line(T, Q1))
    T = pt_add(T, Q1)
    f = _p12_mul(f, line(T, nQ2))
    return _p12_pow(f, (P**12 - 1) // R)


# ----------------------------------------------------------------------------
# KZG decider (snark-verifier/src/pcs/kzg/decider.rs:60-80)
# ----------------------------------------------------------------------------
class DecideError(Exception):
    """Error::AssertionFailure("e(lhs, g2)·e(rhs, -s_g2) == O") (decider.rs:66-67)."""


DECIDE_MSG = "e(lhs, g2)·e(rhs, -s_g2) == O"


def decide_gt(g2, s_g2, lhs, rhs):
    terms = [(lhs, g2_prepare(g2) if g2 is not None else None),
             (rhs, g2_prepare(g2_neg(s_g2)) if s_g2 is not None else None)]
    return final_exponentiation(multi_miller_loop(terms))


def decide(g2, s_g2, lhs, rhs) -> bool:
    return f12_is_one(decide_gt(g2, s_g2, lhs, rhs))


def decide_all(g2, s_g2, accumulators: Sequence[Tuple]) -> int:
    """Returns -1 when every accumulator passes, else the first failing index."""
    assert len(accumulators) > 0  # decider.rs:74
    pg2 = g2_prepare(g2)
    pns = g2_prepare(g2_neg(s_g2))
    for i, (lhs, rhs) in enumerate(accumulators):
        f = final_exponentiation(multi_miller_loop([(lhs, pg2), (rhs, pns)]))
        if not f12_is_one(f):
            return i
    return -1


# ----------------------------------------------------------------------------
# MSM restatements
# ----------------------------------------------------------------------------
def native_msm(scalars: Sequence[int], bases: Sequence) -> Optional[Tuple[int, int]]:
    """NativeLoader::multi_scalar_multiplication (native.rs:61-71). Affine out, None = identity."""
    if len(scalars) == 0:
        raise ValueError("pairs should not be empty")
    acc = (1, 1, 0)
    for s, b in zip(scalars, bases):
        acc = jac_add(acc, jac_mul(jac_from_affine(b), s % R))
    return jac_to_affine(acc)


def window_size(n: int) -> int:
    """msm.rs:247 -- (n as f64).ln().ceil() as usize + 2."""
    return int(math.ceil(math.log(n))) + 2 if n > 0 else 2


def pippenger_serial(scalars: Sequence[int], bases: Sequence, result=(1, 1, 0)):
    """multi_scalar_multiplication_serial (msm.rs:238-283); returns Jacobian."""
    reprs = [(s % R).to_bytes(32, "little") for s in scalars]
    c = window_size(len(scalars))
    num_buckets = (1 << c) - 1
    num_bits = 256

    def windowed(idx, by):
        skip_bits = idx * c
        skip_bytes = skip_bits // 8
        v = int.from_bytes(by[skip_bytes:skip_bytes + 8].ljust(8, b"\0"), "little")
        return (v >> (skip_bits - skip_bytes * 8)) & num_buckets

    num_window = -(-num_bits // c)
    for idx in range(num_window - 1, -1, -1):
        for _ in range(c):
            result = jac_double(result)
        buckets = [None] * num_buckets  # None | ('A', affine) | ('P', jac)
        for by, base in zip(reprs, bases):
            s = windowed(idx, by)
            if s != 0:
                bk = buckets[s - 1]
                if bk is None:
                    buckets[s - 1] = ("A", base)
                elif bk[0] == "A":
                    buckets[s - 1] = ("P", jac_add(jac_from_affine(bk[1]), jac_from_affine(base)))
                else:
                    buckets[s - 1] = ("P", jac_add(bk[1], jac_from_affine(base)))
        running = (1, 1, 0)
        for bk in reversed(buckets):
            if bk is not None:
                running = jac_add(running, jac_from_affine(bk[1]) if bk[0] == "A" else bk[1])
            result = jac_add(result, running)
    return result


def pippenger_msm_parallel(scalars, bases, num_threads: int):
    """msm.rs:287-316 with feature `parallel`: chunk = ceil(n/threads), fold partials."""
    assert len(scalars) == len(bases)
    n = len(scalars)
    if n < num_threads:
        return jac_to_affine(pippenger_serial(scalars, bases))
    chunk = -(-n // num_threads)
    acc = (1, 1, 0)
    for s in range(0, n, chunk):
        acc = jac_add(acc, pippenger_serial(scalars[s:s + chunk], bases[s:s + chunk]))
    return jac_to_affine(acc)


def pippenger_msm(scalars, bases):
    return jac_to_affine(pippenger_serial(scalars, bases))


# ----------------------------------------------------------------------------
# Accumulation (accumulation.rs:146-195, no blind) and limb codec (arithmetic.rs:262-290)
# ----------------------------------------------------------------------------
def powers(r: int, n: int) -> List[int]:
    out = [1]
    for _ in range(n - 1):
        out.append(out[-1] * r % R)
    return out[:n]


def accumulate(accumulators: Sequence[Tuple], r: int):
    pw = powers(r, len(accumulators))
    lhs = native_msm(pw, [a[0] for a in accumulators])
    rhs = native_msm(pw, [a[1] for a in accumulators])
    return lhs, rhs


def create_proof(accumulators: Sequence[Tuple], state: Optional[Sequence[int]] = None):
    """KzgAs::create_proof without blind (snark-verifier/src/pcs/kzg/accumulation.rs:146-195):
    a Poseidon transcript (fresh, or continuing from sponge `state`) absorbs every lhs_i, rhs_i via
    common_ec_point (system/halo2/transcript/halo2.rs:214-226: x, y as Fq -> Fr by fe_to_fe, i.e.
    mod r; the identity has no coordinates -> Error::Transcript), squeezes r (:176), then the two
    r^i MSMs.  Returns ((lhs, rhs), r, the sponge state after the squeeze)."""
    from . import poseidon as op
    sponge = op.Sponge(3, state)
    for a in accumulators:
        op.transcript_common_ec_point(sponge, a[0])
        op.transcript_common_ec_point(sponge, a[1])
    r = sponge.squeeze()
    return accumulate(accumulators, r), r, list(sponge.state)


def fe_to_limbs(x: int, limbs: int = 3, bits: int = 88) -> List[int]:
    mask = (1 << bits) - 1
    return [(x >> (bits * i)) & mask for i in range(limbs)]


def fe_from_limbs(ls: Sequence[int], bits: int = 88, modulus: int = P) -> int:
    """arithmetic.rs:262-274: sum limb_i << (bits * i) (limbs read as canonical ints, no range
    check per limb), then fe_from_big -> from_repr(..).unwrap(): panics when the sum needs more
    than 32 bytes or is >= the modulus."""
    big = sum(int(l) << (bits * i) for i, l in enumerate(ls))
    if big >= 1 << 256 or big >= modulus:
        raise CodecError("fe_from_big: from_repr(..).unwrap() on a non-canonical value")
    return big


# ----------------------------------------------------------------------------
# Codecs on either side of the path
# ----------------------------------------------------------------------------
class CodecError(ValueError):
    pass


POINT_MSG = "Invalid elliptic curve point encoding in proof"


def accumulator_from_limbs(limbs: Sequence[int], n_limbs: int = 3, bits: int = 88):
    """LimbsEncoding<LIMBS, BITS>::from_repr on NativeLoader (pcs/kzg/accumulator.rs:57-77):
    4 * LIMBS Fr limbs -> [lhs_x, lhs_y, rhs_x, rhs_y] via fe_from_limbs, then
    C::from_xy(x, y).unwrap() (on-curve or the (0, 0) identity)."""
    if len(limbs) != 4 * n_limbs:
        raise CodecError("assertion failed: limbs.len() == 4 * LIMBS")
    xs = [fe_from_limbs(limbs[i * n_limbs:(i + 1) * n_limbs], bits) for i in range(4)]
    pts = []
    for x, y in ((xs[0], xs[1]), (xs[2], xs[3])):
        pt = None if (x == 0 and y == 0) else (x, y)
        if pt is not None and not g1_on_curve(pt):
            raise CodecError("C::from_xy(..).unwrap() on a point off the curve")
        pts.append(pt)
    return pts[0], pts[1]


def g1_compress(pt) -> bytes:
    """halo2curves 0.3.1 G1 GroupEncoding::to_bytes (external, restated): x little-endian with the
    parity of y in bit 7 of byte 31; identity = 32 zero bytes.  Parity unpinned (no vectors)."""
    if pt is None:
        return b"\0" * 32
    b = bytearray(int(pt[0]).to_bytes(32, "little"))
    b[31] |= (pt[1] & 1) << 7
    return bytes(b)


def g1_decompress(data: bytes):
    """halo2curves 0.3.1 G1 GroupEncoding::from_bytes (read by PoseidonTranscript::read_ec_point,
    system/halo2/transcript/halo2.rs:247-260): clear the sign bit, x must be canonical; x == 0 with
    sign 0 is the identity; otherwise y = sqrt(x^3 + 3) (none -> error), negated when its parity
    differs from the sign bit."""
    if len(data) != 32:
        raise CodecError(POINT_MSG)
    sign = data[31] >> 7
    x = int.from_bytes(bytes(data[:31]) + bytes([data[31] & 0x7F]), "little")
    if x >= P:
        raise CodecError(POINT_MSG)
    if x == 0 and sign == 0:
        return None
    y = sqrt_fp((x * x * x + B) % P)
    if y is None:
        raise CodecError(POINT_MSG)
    if (y & 1) != sign:
        y = (P - y) % P
    return (x, y)


def g1_evm_encode(pt) -> bytes:
    """EvmTranscript point encoding: x || y, 32-byte big-endian each (transcript/evm.rs:223-242)."""
    if pt is None:
        return b"\0" * 64
    return int(pt[0]).to_bytes(32, "big") + int(pt[1]).to_bytes(32, "big")


def g1_evm_decode(data: bytes):
    """EvmTranscript::read_ec_point (transcript/evm.rs:223-242): both coordinates from_repr
    (canonical, < p), then C::from_xy (on-curve, or (0, 0) = identity)."""
    if len(data) != 64:
        raise CodecError(POINT_MSG)
    x = int.from_bytes(data[:32], "big")
    y = int.from_bytes(data[32:], "big")
    if x >= P or y >= P:
        raise CodecError(POINT_MSG)
    if x == 0 and y == 0:
        return None
    if not g1_on_curve((x, y)):
        raise CodecError(POINT_MSG)
    return (x, y)


def _g2_words(q) -> bytes:
    (x0, x1), (y0, y1) = q
    return b"".join(int(v).to_bytes(32, "big") for v in (x1, x0, y1, y0))


def eip197_input(g2, s_g2, lhs, rhs) -> bytes:
    """The 0x180-byte ecPairing (EIP-197) input the EVM decider builds (pcs/kzg/decider.rs:
    107-127, loader/evm/loader.rs:338-382): lhs, g2, rhs, -s_g2; G2 words (x.c1, x.c0, y.c1, y.c0)."""
    return g1_evm_encode(lhs) + _g2_words(g2) + g1_evm_encode(rhs) + _g2_words(g2_neg(s_g2))


def eip197_parse(data: bytes):
    """Inverse of eip197_input: (lhs, g2, rhs, minus_s_g2)."""
    if len(data) != 0x180:
        raise CodecError("EIP-197 input must be 0x180 bytes per pairing check")

    def g2_at(o):
        w = [int.from_bytes(data[o + 32 * i:o + 32 * (i + 1)], "big") for i in range(4)]
        return ((w[1], w[0]), (w[3], w[2]))
    return g1_evm_decode(data[0:64]), g2_at(64), g1_evm_decode(data[192:256]), g2_at(256)


# ----------------------------------------------------------------------------
# Encodings (C-ABI layout): 4 x u64 little-endian limbs; Montgomery or canonical
# ----------------------------------------------------------------------------
def to_mont(x: int, m: int = P) -> int:
    return (x << 256) % m


def from_mont(x: int, m: int = P) -> int:
    return x * inv(1 << 256, m) % m


def fe_bytes(x: int) -> bytes:
    return int(x).to_bytes(32, "little")


def g1_bytes(pt, mont: bool = False) -> bytes:
    if pt is None:
        return b"\0" * 64
    x, y = pt
    if mont:
        x, y = to_mont(x), to_mont(y)
    return fe_bytes(x) + fe_bytes(y)


def g1_from_bytes(b: bytes, mont: bool = False):
    x = int.from_bytes(b[:32], "little")
    y = int.from_bytes(b[32:64], "little")
    if x == 0 and y == 0:
        return None
    if mont:
        x, y = from_mont(x), from_mont(y)
    return (x, y)


def g2_bytes(q, mont: bool = False) -> bytes:
    if q is None:
        return b"\0" * 128
    out = b""
    for c in (q[0][0], q[0][1], q[1][0], q[1][1]):
        out += fe_bytes(to_mont(c) if mont else c)
    return out


# ----------------------------------------------------------------------------
# Deterministic synthetic inputs, index-addressable so the
# C++ oracle and the device generator reproduce identical bytes:
#   state_i = seed * 0x9E3779B97F4A7C15 + i * 0xD1B54A32D192ED03  (mod 2^64)
#   then SplitMix64 draws from state_i.
# ----------------------------------------------------------------------------
M64 = (1 << 64) - 1
GOLDEN = 0x9E3779B97F4A7C15
STREAM = 0xD1B54A32D192ED03


class SplitMix64:
    def __init__(self, state: int):
        self.s = state & M64

    def next(self) -> int:
        self.s = (self.s + GOLDEN) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)


def stream_for(seed: int, i: int) -> SplitMix64:
    return SplitMix64((seed * GOLDEN + i * STREAM) & M64)


def _draw254(sm: SplitMix64) -> int:
    l = [sm.next() for _ in range(4)]
    l[3] &= (1 << 62) - 1
    return l[0] | (l[1] << 64) | (l[2] << 128) | (l[3] << 192)


def gen_scalar(seed: int, i: int) -> int:
    sm = stream_for(seed, i)
    while True:
        v = _draw254(sm)
        if v < R:
            return v


def gen_base(seed: int, i: int):
    sm = stream_for(seed, i)
    while True:
        x = _draw254(sm)
        if x >= P:
            continue
        y = sqrt_fp(x * x * x + B)
        if y is None:
            continue
        if (sm.next() & 1) != (y & 1):
            y = P - y
        return (x, y)


def gen_scalars(seed: int, n: int, start: int = 0) -> List[int]:
    return [gen_scalar(seed, start + i) for i in range(n)]


def gen_bases(seed: int, n: int, start: int = 0) -> List:
    return [gen_base(seed, start + i) for i in range(n)]


SEED_SCALARS = 0x5CA1A75
SEED_BASES = 0xBA5E5
SEED_TRAPDOOR = 0xD3C1DE


def gen_decider_case(n: int, seed: int = SEED_TRAPDOOR, bad: Sequence[int] = (), start: int = 0):
    """dk = (G1, G2, s G2); acc_i = (s t_i G1, t_i G1) with t_i the seeded scalar start + i (every
    accumulator distinct); lhs_k += G1 for k in `bad`."""
    s = gen_scalar(seed, 0)
    s_g2 = g2_mul(G2_GEN, s)
    accs = []
    for i in range(n):
        t = gen_scalar(seed, 1 + start + i)
        rhs = g1_mul(G1_GEN, t)
        lhs = g1_mul(G1_GEN, s * t % R)
        if i in bad:
            lhs = g1_add(lhs, G1_GEN)
        accs.append((lhs, rhs))
    return G2_GEN, s_g2, accs
