"""GPU Poseidon through the C ABI: the reference's own permutation KATs
(poseidon/tests.rs:34-85), random states against the oracle permutation, and the sponge /
transcript against the oracle's restatement of poseidon.rs:412-467 (sponge level: parity
unpinned beyond that restatement -- the reference holds no sponge vectors)."""
import random

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import bn254 as b
from oracle import poseidon as op

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("key", ["perm_x5_254_3", "perm_x5_254_5"])
def test_permutation_kat(gpu, key):
    from svgpu import poseidon as gp
    k = load_golden("poseidon_kat.json")[key]
    out = gp.permute([[int(v) for v in k["input"]]], t=k["t"])
    assert out == [[int(v) for v in k["output"]]]


@pytest.mark.parametrize("t", [3, 5])
def test_permutation_random_both_forms(gpu, t):
    import svgpu
    from svgpu import _lib, device as dv, encoding as enc
    rng = random.Random(7 + t)
    states = [[rng.randrange(b.R) for _ in range(t)] for _ in range(40)]
    states[0] = [0] * t
    states[1] = [b.R - 1] * t
    want = [op.permutation(s, t, *op.PARAMS[t]) for s in states]
    from svgpu import poseidon as gp
    assert gp.permute(states, t) == want
    # device entry point, Montgomery in HBM
    flat = [v for s in states for v in s]
    buf = torch.from_numpy(enc.scalars_array(flat, svgpu.SV_MONTGOMERY).view(np.int64)).to(gpu)
    dv.poseidon_permute(buf, t, _lib.SV_MONTGOMERY)
    torch.cuda.synchronize()
    got = [enc._from_form(enc.limbs_to_int(r), b.R, _lib.SV_MONTGOMERY) for r in buf.cpu().numpy().view(np.uint64)]
    assert got == [v for s in want for v in s]


@pytest.mark.parametrize("t", [3, 5])
def test_sponge_squeeze_lengths_and_continuation(gpu, t):
    from svgpu import poseidon as gp
    rng = random.Random(100 + t)
    for length in range(0, 3 * t + 2):
        ref = op.Sponge(t)
        dev = gp.Poseidon(t)
        for round_ in range(3):  # squeezes continue from the previous state, like a transcript
            els = [rng.randrange(b.R) for _ in range(length + round_)]
            ref.update(els)
            dev.update(els)
            assert dev.squeeze() == ref.squeeze(), (length, round_)
            assert dev.state == ref.state
    dev.clear()
    assert dev.state == gp.Poseidon.default_state(t) and dev.buf == []


def test_squeeze_many_ragged_batch(gpu):
    from svgpu import poseidon as gp
    rng = random.Random(5)
    lens = [0, 1, 2, 3, 4, 7, 0, 11, 2, 64]
    refs, devs = [], []
    for L in lens:
        els = [rng.randrange(b.R) for _ in range(L)]
        r, d = op.Sponge(3), gp.Poseidon(3)
        r.update(els)
        d.update(els)
        refs.append(r)
        devs.append(d)
    assert gp.squeeze_many(devs) == [r.squeeze() for r in refs]
    assert [d.state for d in devs] == [r.state for r in refs]


def test_transcript_challenges(gpu):
    from svgpu import poseidon as gp
    pts = [b.g1_mul(b.G1_GEN, k) for k in (1, 2, 12345, b.R - 1)]
    tr = gp.PoseidonTranscript()
    ref = op.Sponge(3)
    for i, p in enumerate(pts):
        tr.common_ec_point(p)
        op.transcript_common_ec_point(ref, p)
        tr.common_scalar(i * 7919)
        ref.update([i * 7919])
        assert tr.squeeze_challenge() == ref.squeeze()
    with pytest.raises(ValueError, match="Invalid elliptic curve point"):
        tr.common_ec_point(None)


def test_device_batch_of_identical_transcripts(gpu):
    """2^16 sponges in one launch: every lane absorbs the same 9 elements -> one value, equal to
    the oracle's (size-independent property + spot parity)."""
    import svgpu
    from svgpu import device as dv, encoding as enc
    n, L, t = 1 << 16, 9, 3
    rng = random.Random(11)
    els = [rng.randrange(b.R) for _ in range(L)]
    ref = op.Sponge(t)
    ref.update(els)
    want = ref.squeeze()
    mont = svgpu.SV_MONTGOMERY
    st0 = torch.from_numpy(enc.scalars_array(op.Sponge(t).state, mont).view(np.int64)).to(gpu)
    states = st0.repeat(n, 1).contiguous()
    e1 = torch.from_numpy(enc.scalars_array(els, mont).view(np.int64)).to(gpu)
    elements = e1.repeat(n, 1).contiguous()
    offsets = torch.arange(0, (n + 1) * L, L, dtype=torch.int64, device=gpu)
    out = dv.poseidon_squeeze(states, elements, offsets, t, mont)
    torch.cuda.synchronize()
    o = out.cpu().numpy().view(np.uint64)
    assert (o == o[0]).all()
    assert enc._from_form(enc.limbs_to_int(o[0]), b.R, mont) == want
