"""The 29-bit-limb field and XYZZ mixed addition (csrc/field29.hpp, csrc/curve29.hpp), run on the
host through tests/native/field29check.cpp and checked with Python integers: every operation's
value mod p and its stated output bound, and madd against the oracle's affine group law
(oracle/bn254.py), including the identity, doubling (through the addition's own products) and P + (-P) branches.  CPU only."""
import os
import random
import subprocess

import pytest

from oracle import bn254 as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
P = ob.P
RP = (1 << 261) % P  # R' = 2^261
RINV = pow(RP, -1, P)


@pytest.fixture(scope="module", params=["field29check", "field29check_asan"])
def f29(request):
    """The harness as built, and again under ASan + UBSan (any report fails the run)."""
    r = subprocess.run(["make", "-s", "-C", NATIVE, "build/" + request.param], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(NATIVE, "build", request.param)


def _limbs(h):
    """The harness prints a value as its 9 limbs, most significant first, 8 hex digits each."""
    if len(h) != 72:
        return int(h, 16)
    return sum(int(h[8 * i:8 * i + 8], 16) << (29 * (8 - i)) for i in range(9))


@pytest.mark.parametrize("field", ["fq", "fr"])
def test_field_ops_values_and_bounds(f29, field):
    """Every operation over both moduli (FqM29 = p for the bucket chain, FrM29 = r for Poseidon)."""
    P = ob.P if field == "fq" else ob.R  # noqa: N806 (the modulus of this run)
    RINV = pow((1 << 261) % P, -1, P)  # noqa: N806
    args = [f29] if field == "fq" else [f29, "fr"]
    out = subprocess.run(args, capture_output=True, text=True, check=True).stdout
    counts = {}
    for line in out.splitlines():
        f = line.split()
        op, v = f[0], [_limbs(x) for x in f[1:]]
        counts[op] = counts.get(op, 0) + 1
        if op == "mul_sum3":
            a0, b0, a1, b1, a2, b2, r = v
            if any(x >= 9 * P for x in (a0, a1, a2)) or any(x >= P for x in (b0, b1, b2)):
                continue
            assert r < 2 * P, line
            assert r % P == (a0 * b0 + a1 * b1 + a2 * b2) * RINV % P, line
        elif op in ("mul", "mul_ilp", "sqr", "mul_sum2"):
            bound_in = 12 * P if op != "mul_sum2" else 9 * P
            ins, r = v[:-1], v[-1]
            if any(x >= bound_in for x in ins):
                continue  # outside the stated contract: not checked
            if op in ("mul", "mul_ilp"):
                want = ins[0] * ins[1]
            elif op == "sqr":
                want = ins[0] * ins[0]
            else:
                want = ins[0] * ins[1] + ins[2] * ins[3]
            assert r < 2 * P, line
            assert r % P == want * RINV % P, line
        elif op == "mul_sub8":
            a, b, c, r = v
            if a >= 12 * P or b >= 12 * P or c >= 8 * P:
                continue
            assert 0 <= r < 10 * P and r % P == (a * b * RINV - c) % P, line
        elif op == "sqr_sub2c6":
            a, b, c, r = v
            if a >= 12 * P or b >= 2 * P or c >= 2 * P:
                continue
            assert 0 < r < 8 * P and r % P == (a * a * RINV - b - 2 * c) % P, line
        elif op == "sub2c6":
            a, b, c, r = v
            want = a + 6 * P - b - 2 * c
            if not 0 <= want < (1 << 261):
                continue  # outside the stated contract: not checked
            assert r == want, line
        elif op.startswith("sub"):
            k = int(op[3:])
            a, b, r = v
            if b >= k * P:
                continue
            assert r == a - b + k * P, line
        elif op == "add":
            a, b, r = v
            assert r == a + b, line
        elif op.startswith("csub"):
            k = int(op[4:])
            a, r = v
            if a >= 2 * k * P:
                continue
            assert r % P == a % P and r < k * P, line
        elif op in ("zero6", "zero10", "zero16"):
            a, z = v
            if a >= int(op[4:]) * P:
                continue
            assert z == (1 if a % P == 0 else 0), line
        elif op == "words":
            a, back = v
            if a < (1 << 256):
                assert back == a, line
        elif op == "to_r29":
            a, r29, back = v
            assert r29 < 2 * P and r29 % P == a * 32 % P and back == a, line
        elif op == "to_r32":
            a, r = v
            assert r < P and r == a * pow(32, -1, P) % P, line
    assert counts.get("mul", 0) >= 3000 and counts.get("mul_ilp", 0) >= 3000 and counts.get("to_r32", 0) >= 3000 and counts.get("mul_sum3", 0) >= 3000
    assert counts.get("zero6", 0) >= (3006 if field == "fq" else 0)
    assert counts.get("zero10", 0) >= (3010 if field == "fq" else 0)
    assert counts.get("zero16", 0) >= (3016 + 31 if field == "fq" else 0)  # every multiple k p, k < 16
    assert counts.get("sub2c6", 0) >= 3000 and counts.get("sub8", 0) >= 3000
    assert counts.get("mul_sub8", 0) >= 3000 and counts.get("sqr_sub2c6", 0) >= 3000


def _state(pt, rng, identity=False, xmax=4):
    """A random XYZZ representation of an affine point inside the stated bounds (R' form)."""
    if identity:
        return (0, 0, 0, 0)
    x, y = pt
    z = rng.randrange(1, P)
    zz, zzz = z * z % P, z * z * z % P
    X, Y = x * zz % P, y * zzz % P
    m = lambda v: v * RP % P  # noqa: E731
    return (m(X) + rng.randrange(xmax) * P, m(Y) + rng.randrange(2) * P, m(zz) + rng.randrange(2) * P,
            m(zzz) + rng.randrange(2) * P)


def _to_affine(X, Y, ZZ, ZZZ):
    X, Y, ZZ, ZZZ = (v * RINV % P for v in (X, Y, ZZ, ZZZ))
    if ZZ == 0:
        return None
    return (X * pow(ZZ, -1, P) % P, Y * pow(ZZZ, -1, P) % P)


@pytest.mark.parametrize("live", [False, True])
@pytest.mark.parametrize("neg", [False, True])
def test_madd_group_law(f29, neg, live):
    """state + (x2, +-y2): the chain's signed point (neg folds the sign into S2 = y2 ZZZ)."""
    rng = random.Random(29 + neg)
    g = (1, 2)
    cases = []  # (state, x2, y2, expected affine sum or None)
    for n in range(300):
        a = ob.g1_mul(g, rng.randrange(1, ob.R))
        b = ob.g1_mul(g, rng.randrange(1, ob.R))
        kind = n % 10
        if kind == 7:
            b = a  # doubling branch
        elif kind == 8:
            b = ob.g1_neg(a)  # P + (-P)
        st = _state(a, rng, identity=(kind == 9), xmax=8)  # madd's chain state: X below 8p
        want = b if kind == 9 else ob.g1_add(a, b)
        yv = ob.g1_neg(b)[1] if neg else b[1]  # the point handed over is (x, y) with y negated by neg
        xb = b[0] * RP % P + rng.randrange(2) * P
        yb = yv * RP % P + rng.randrange(2) * P
        cases.append((st, xb, yb, want))
    inp = "\n".join(" ".join(hex(v) for v in (*st, xb, yb)) for st, xb, yb, _ in cases) + "\n"
    mode = ("maddl" if live else "madd") + ("n" if neg else "")  # live: start / madd_live (round 6)
    out = subprocess.run([f29, mode], input=inp, capture_output=True, text=True,
                         check=True).stdout.splitlines()
    assert len(out) == len(cases)
    for (st, xb, yb, want), line in zip(cases, out):
        X, Y, ZZ, ZZZ = (_limbs(v) for v in line.split())
        assert X < 8 * P and Y < 2 * P and ZZ < 2 * P and ZZZ < 2 * P, line  # madd's chain: X < 8p
        got = _to_affine(X, Y, ZZ, ZZZ)
        assert got == (None if want is None else tuple(want)), (st, xb, yb)
        if got is None and live:
            assert ZZ == 0, line  # a cancelled chain reads as the identity by ZZ == 0 alone
        elif got is None:
            assert X == Y == ZZ == ZZZ == 0, line  # the identity is exactly zero limbs


def test_xyzz_add_group_law(f29):
    """The full XYZZ addition (k_wsum_tree's running sums): random representations of both points
    within the stated bounds, the identity on either side, doubling (p = q, also in different
    representations) and p + (-p)."""
    rng = random.Random(31)
    g = (1, 2)
    cases = []
    for n in range(300):
        a = ob.g1_mul(g, rng.randrange(1, ob.R))
        b = ob.g1_mul(g, rng.randrange(1, ob.R))
        kind = n % 10
        if kind == 6:
            b = a
        elif kind == 7:
            b = ob.g1_neg(a)
        sa = _state(a, rng, identity=(kind == 8))
        sb = _state(b, rng, identity=(kind == 9))
        pa = None if kind == 8 else a
        pb = None if kind == 9 else b
        want = pb if pa is None else (pa if pb is None else ob.g1_add(pa, pb))
        cases.append((sa, sb, want))
    inp = "\n".join(" ".join(hex(v) for v in (*sa, *sb)) for sa, sb, _ in cases) + "\n"
    out = subprocess.run([f29, "xadd"], input=inp, capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == len(cases)
    for (sa, sb, want), line in zip(cases, out):
        X, Y, ZZ, ZZZ = (_limbs(v) for v in line.split())
        assert X < 4 * P and Y < 2 * P and ZZ < 2 * P and ZZZ < 2 * P, line
        got = _to_affine(X, Y, ZZ, ZZZ)
        assert got == (None if want is None else tuple(want)), (sa, sb)
        if got is None:
            assert X == Y == ZZ == ZZZ == 0, line
