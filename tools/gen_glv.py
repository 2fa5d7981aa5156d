"""Derive the BN254 GLV constants used by snark-verifier-axiom_amd/csrc/glv.hpp and check them.

lambda: the cube root of unity mod r whose endomorphism is phi(x, y) = (beta x, y) on G1;
(a1, -B1), (a2, b2): reduced lattice basis of {(x, y) : x + y lambda = 0 mod r} (GLV, extended Euclid);
g1 = floor(2^256 b2 / r), g2 = floor(2^256 B1 / r) for the Babai rounding.
usage: python3 tools/gen_glv.py   (prints the limb tables; asserts the identities)
"""
import math
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import bn254 as ob  # noqa: E402

r, p = ob.R, ob.P
LAMBDA = 0xB3C4D79D41A917585BFC41088D8DAAA78B17EA66B99C90DD
BETA = 0x59E26BCEA0D48BACD4F263F1ACDB5C4F5763473177FFFFFE


def basis(n, lam):
    s0, t0, r0, s1, t1, r1 = 1, 0, n, 0, 1, lam
    rows = [(r0, t0), (r1, t1)]
    while r1:
        q = r0 // r1
        r0, r1 = r1, r0 - q * r1
        t0, t1 = t1, t0 - q * t1
        rows.append((r1, t1))
    m = max(i for i, (ri, _) in enumerate(rows) if ri >= math.isqrt(n))
    (ra, ta), (rb, tb), (rc, tc) = rows[m], rows[m + 1], rows[m + 2]
    v1 = (rb, -tb)
    v2 = (ra, -ta) if ra * ra + ta * ta <= rc * rc + tc * tc else (rc, -tc)
    return v1, v2


def constants():
    assert pow(LAMBDA, 3, r) == 1 and LAMBDA != 1 and pow(BETA, 3, p) == 1 and BETA != 1
    g = ob.G1_GEN
    assert ob.g1_eq(ob.g1_mul(g, LAMBDA), ((BETA * g[0]) % p, g[1])), "beta does not match lambda"
    (a1, b1), (a2, b2) = basis(r, LAMBDA)
    assert (a1 + b1 * LAMBDA) % r == 0 and (a2 + b2 * LAMBDA) % r == 0
    B1 = -b1
    assert B1 > 0 and b2 > 0 and a1 == b2 and a1 * b2 + a2 * B1 == r
    g1, g2 = (b2 << 256) // r, (B1 << 256) // r
    assert 3 * (a1 + a2) // 4 < 2**127 and 3 * (B1 + b2) // 4 < 2**127
    return dict(beta_mont=BETA * ob.RP % p, g1=g1, g2=g2, a1=a1, a2=a2, b1=B1)


def split(k, c=None):
    c = c or constants()
    c1 = (k * c["g1"] + (1 << 255)) >> 256
    c2 = (k * c["g2"] + (1 << 255)) >> 256
    return k - c1 * c["a1"] - c2 * c["a2"], c1 * c["b1"] - c2 * c["a1"]


def limbs(v, n=None):
    n = n or (v.bit_length() + 31) // 32
    return "{" + ", ".join("0x%08xu" % ((v >> (32 * i)) & 0xFFFFFFFF) for i in range(n)) + "}"


if __name__ == "__main__":
    c = constants()
    for k in [0, 1, r - 1] + [random.randrange(r) for _ in range(20000)]:
        k1, k2 = split(k, c)
        assert (k1 + k2 * LAMBDA - k) % r == 0 and abs(k1) < 2**127 and abs(k2) < 2**127
    print("GLV_BETA_MONT", limbs(c["beta_mont"], 8))
    for name in ("g1", "g2", "a1", "a2", "b1"):
        print("GLV_" + name.upper(), limbs(c[name]))
