"""The product's host Poseidon transcript (csrc/host_poseidon.hpp: the serial sponge of
sv_bn254_kzg_create_proof) against oracle/poseidon.py (pinned by the reference KATs,
poseidon/tests.rs:34-85): fresh and continued sponges, every buffer length parity (the padded
short chunk and the extra permutation of an exact buffer, poseidon.rs:455-467).  CPU only."""
import os
import random
import subprocess

import pytest

from oracle import poseidon as op

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


@pytest.fixture(scope="module", params=["host_sponge", "host_sponge_asan"])
def sponge_bin(request):
    """The harness as built, and again under ASan + UBSan (any report fails the run)."""
    r = subprocess.run(["make", "-s", "-C", NATIVE, "build/" + request.param], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(NATIVE, "build", request.param)


def _run(binary, state, elements):
    inp = ("-" if state is None else " ".join(hex(v) for v in state)) + "\n" + "\n".join(hex(e) for e in elements)
    out = subprocess.run([binary], input=inp, capture_output=True, text=True, check=True).stdout.split()
    return int(out[0], 16), [int(v, 16) for v in out[1:4]]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 7, 128, 257])
def test_host_sponge_matches_oracle(sponge_bin, n):
    rng = random.Random(n)
    els = [rng.randrange(op.FR_MODULUS) for _ in range(n)]
    sp = op.Sponge(3)
    sp.update(els)
    r = sp.squeeze()
    assert _run(sponge_bin, None, els) == (r, sp.state)


def test_host_sponge_continues_state(sponge_bin):
    rng = random.Random(99)
    state = [rng.randrange(op.FR_MODULUS) for _ in range(3)]
    els = [op.FR_MODULUS - 1, 0, 1, rng.randrange(op.FR_MODULUS), 5]
    sp = op.Sponge(3, state)
    sp.update(els)
    r = sp.squeeze()
    assert _run(sponge_bin, state, els) == (r, sp.state)
