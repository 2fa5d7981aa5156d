"""The 29-bit-limb Poseidon constants (poseidon_consts.hpp *_R29_INIT, tools/gen_consts.py) are the
same constants as the 8 x 32-bit Montgomery ones: c 2^261 = 32 (c 2^256) mod r, limbs normalized.
CPU only."""
import os
import re

import pytest

from oracle import bn254 as ob

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "snark-verifier-axiom_amd", "csrc", "poseidon_consts.hpp")


def _macro(text, name):
    m = re.search(r"#define %s \{([^}]*)\}" % name, text)
    assert m, name
    return [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",")]


@pytest.mark.parametrize("key", ["START", "PARTIAL", "END", "MDS", "PRE", "SPARSE"])
def test_r29_constants_match(key):
    text = open(HDR).read()
    w32 = _macro(text, "SV_POSEIDON_T3_%s_INIT" % key)
    w29 = _macro(text, "SV_POSEIDON_T3_%s_R29_INIT" % key)
    assert len(w32) % 8 == 0 and len(w29) == len(w32) // 8 * 9
    r = ob.R
    for k in range(len(w32) // 8):
        v32 = sum(w << (32 * i) for i, w in enumerate(w32[8 * k:8 * k + 8]))
        limbs = w29[9 * k:9 * k + 9]
        assert all(x < (1 << 29) for x in limbs)
        v29 = sum(x << (29 * i) for i, x in enumerate(limbs))
        assert v32 < r and v29 < r and v29 == v32 * 32 % r, (key, k)
