"""Device paths of the fused field primitives (csrc/field.hpp fe_sqr_hp / fe_mul_sum<N>,
csrc/curve.hpp mul_diff) on edge operands, against Python big-int Montgomery arithmetic.

Their inline-asm device code differs from the host build (which falls back to a*a and separate
products) and the MSM / Poseidon parity tests only reach them with random operands; this hits
the boundary cases of the one-reduction bound: 0, 1, p-1, p-2, 2^k, all-ones low limbs, and
the N = 3 worst case near 1.75 p that needs the final conditional subtraction.  Harness:
tests/native/fieldcheck.hip (test-only, built by __graft_entry__.build()).
"""
import ctypes
import os
import random

import numpy as np
import pytest

from conftest import ROOT
from oracle import bn254 as b

pytestmark = pytest.mark.gpu

LIB = os.path.join(ROOT, "tests", "native", "build", "libfieldcheck.so")
MODS = {0: b.P, 1: b.R}
OP_MUL, OP_SQR_HP, OP_SUM1, OP_SUM2, OP_SUM3, OP_MUL_DIFF = range(6)


def _edges(p):
    v = [0, 1, 2, p - 1, p - 2, p - 3, (p - 1) // 2, (p + 1) // 2, (1 << 253), (1 << 253) - 1, p >> 1]
    v += [1 << k for k in range(0, 254, 17)]
    v += [(1 << (32 * k)) - 1 for k in range(1, 8)]             # all-ones low limbs
    v += [p - ((1 << (32 * k)) - 1) for k in range(1, 7)]       # just below p, ragged low limbs
    v += [(p - 1) ^ ((1 << 32) - 1)]
    rng = random.Random(0xF1E1D)
    v += [rng.randrange(p) for _ in range(24)]
    return [x % p for x in v]


def _arr(vals):
    out = np.zeros((len(vals), 8), np.uint32)
    for i, x in enumerate(vals):
        for k in range(8):
            out[i, k] = (x >> (32 * k)) & 0xFFFFFFFF
    return out


def _ints(a):
    return [sum(int(r[k]) << (32 * k) for k in range(8)) for r in a]


@pytest.fixture(scope="module")
def fc():
    assert os.path.exists(LIB), "tests/native/build/libfieldcheck.so missing: run __graft_entry__.build()"
    lib = ctypes.CDLL(LIB)
    lib.fc_run.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 5 + [ctypes.c_size_t]
    lib.fc_run.restype = ctypes.c_int
    return lib


def _run(fc, op, field, A, B, C, D):
    arrs = [_arr(x) for x in (A, B, C, D)]
    out = np.zeros_like(arrs[0])
    rc = fc.fc_run(op, field, *[x.ctypes.data for x in arrs], out.ctypes.data, len(A))
    assert rc == 0, f"fc_run hip error {rc}"
    return _ints(out)


@pytest.mark.parametrize("field", [0, 1], ids=["Fq", "Fr"])
def test_fused_primitives_on_edges(gpu, fc, field):
    p = MODS[field]
    rinv = pow(1 << 256, -1, p)
    E = _edges(p)
    # all ordered pairs of edge values for the products; c, d shifted copies for the sums
    A = [x for x in E for _ in E]
    B = [y for _ in E for y in E]
    C = B[7:] + B[:7]
    D = A[13:] + A[:13]
    mont = lambda x, y: x * y * rinv % p  # noqa: E731
    assert _run(fc, OP_MUL, field, A, B, C, D) == [mont(x, y) for x, y in zip(A, B)]
    assert _run(fc, OP_SQR_HP, field, A, B, C, D) == [mont(x, x) for x in A]
    assert _run(fc, OP_SUM1, field, A, B, C, D) == [mont(x, y) for x, y in zip(A, B)]
    assert _run(fc, OP_SUM2, field, A, B, C, D) == [(x * y + z * w) * rinv % p for x, y, z, w in zip(A, B, C, D)]
    assert _run(fc, OP_SUM3, field, A, B, C, D) == [(x * y + z * w + y * z) * rinv % p
                                                    for x, y, z, w in zip(A, B, C, D)]
    if field == 0:
        assert _run(fc, OP_MUL_DIFF, field, A, B, C, D) == [(x * y - z * w) * rinv % p
                                                            for x, y, z, w in zip(A, B, C, D)]


@pytest.mark.parametrize("field", [0, 1], ids=["Fq", "Fr"])
def test_sum3_worst_case_needs_final_subtraction(gpu, fc, field):
    """Three products of (p-1)^2 scan to just under the 2p bound: the result must still be reduced."""
    p = MODS[field]
    rinv = pow(1 << 256, -1, p)
    top = [p - 1, p - 2, p - 1 - (1 << 200), p - ((1 << 64) - 1)]
    A = [x for x in top for _ in top]
    B = [y for _ in top for y in top]
    got = _run(fc, OP_SUM3, field, A, B, B, A)
    exp = [(x * y + y * x + y * y) * rinv % p for x, y in zip(A, B)]
    assert got == exp
    assert all(g < p for g in got)
