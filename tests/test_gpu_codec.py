"""Device codecs through the C ABI against the oracle restatements:
compressed and EVM point decoding (valid, identity, every invalid class), LimbsEncoding
from_repr, and EIP-197 records decided on the GPU.  The compressed layout is halo2curves'
(external): parity unpinned beyond the oracle restatement."""
import random

import numpy as np
import pytest

from conftest import pt, q2
from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def _points(k, seed=1):
    rng = random.Random(seed)
    return [b.g1_mul(b.G1_GEN, rng.randrange(1, b.R)) for _ in range(k)]


def test_decode_compressed(gpu):
    from svgpu import codec
    pts = _points(300) + [None, b.g1_neg(b.G1_GEN), b.G1_GEN]
    data = b"".join(b.g1_compress(p) for p in pts)
    assert codec.read_ec_points(data) == [b.g1_decompress(b.g1_compress(p)) for p in pts] == pts


def test_decode_compressed_invalid(gpu):
    from svgpu import codec
    good = [b.g1_compress(p) for p in _points(10, 2)]
    bad_x = next(x for x in range(1, 100) if b.sqrt_fp((x ** 3 + 3) % b.P) is None)
    cases = {
        "x_ge_p": (b.P + 1).to_bytes(32, "little"),
        "no_sqrt": bad_x.to_bytes(32, "little"),
        "no_sqrt_signed": bytes(bytearray(bad_x.to_bytes(32, "little"))[:31]) + bytes([0x80]),
    }
    for name, enc_bad in cases.items():
        data = b"".join(good[:7]) + enc_bad + b"".join(good[7:])
        with pytest.raises(codec.TranscriptError, match="Invalid elliptic curve point encoding in proof") as ei:
            codec.read_ec_points(data)
        assert ei.value.index == 7, name
        with pytest.raises(b.CodecError):
            b.g1_decompress(enc_bad)


def test_decode_evm(gpu):
    from svgpu import _lib, codec
    pts = _points(257, 3) + [None]
    data = b"".join(b.g1_evm_encode(p) for p in pts)
    assert codec.read_ec_points(data, _lib.SV_ENC_EVM) == pts
    for bad in ((b.P).to_bytes(32, "big") + (2).to_bytes(32, "big"),
                (1).to_bytes(32, "big") + (3).to_bytes(32, "big"),
                (0).to_bytes(32, "big") + (1).to_bytes(32, "big")):
        with pytest.raises(codec.TranscriptError) as ei:
            codec.read_ec_points(data[:64 * 5] + bad + data[64 * 5:], _lib.SV_ENC_EVM)
        assert ei.value.index == 5


def test_limbs_encoding(gpu):
    import svgpu
    from svgpu import codec
    accs = [(p, q) for p, q in zip(_points(40, 4), _points(40, 5))] + [(None, None), (b.G1_GEN, None)]
    reprs = [sum((b.fe_to_limbs(c) for c in ((l or (0, 0))[0], (l or (0, 0))[1], (r or (0, 0))[0],
                                             (r or (0, 0))[1])), []) for l, r in accs]
    got = codec.LimbsEncoding(3, 88).from_repr_many(reprs)
    assert [(a.lhs, a.rhs) for a in got] == [b.accumulator_from_limbs(r) for r in reprs] == accs
    # overlapping limbs are summed exactly like fe_from_limbs (no per-limb range check)
    x = accs[0][0][0]
    over = [x - (5 << 88), 5, 0]
    r = over + b.fe_to_limbs(accs[0][0][1]) + reprs[0][6:]
    assert codec.LimbsEncoding().from_repr(r).lhs == accs[0][0]
    # off-curve / non-canonical -> the reference's unwrap panic, lowest bad accumulator reported
    bad = list(reprs)
    bad[3] = reprs[3][:-1] + [reprs[3][-1] ^ 1]
    bad[9] = [0, 0, 1 << 90] + reprs[9][3:]
    with pytest.raises(svgpu.ReferencePanic, match="accumulator 3"):
        codec.LimbsEncoding().from_repr_many(bad)


def test_decide_eip197(gpu, golden_decider):
    import svgpu
    from svgpu import codec
    for c in golden_decider["cases"]:
        dk = svgpu.KzgDecidingKey(b.G1_GEN, q2(c["g2"]), q2(c["s_g2"]))
        accs = [svgpu.KzgAccumulator(pt(l), pt(r)) for l, r in zip(c["lhs"], c["rhs"])]
        recs = b"".join(codec.eip197_input(dk, a) for a in accs)
        assert recs == b"".join(b.eip197_input(dk.g2, dk.s_g2, a.lhs, a.rhs) for a in accs)
        assert codec.decide_eip197(recs) == c["first_fail"], c["name"]
    # an invalid G1 word fails that check (the precompile would revert)
    c = next(c for c in golden_decider["cases"] if c["first_fail"] < 0 and len(c["lhs"]) > 3)
    dk = svgpu.KzgDecidingKey(b.G1_GEN, q2(c["g2"]), q2(c["s_g2"]))
    accs = [svgpu.KzgAccumulator(pt(l), pt(r)) for l, r in zip(c["lhs"], c["rhs"])]
    recs = bytearray(b"".join(codec.eip197_input(dk, a) for a in accs))
    recs[2 * 0x180 + 192 + 63] ^= 1  # rhs.y of check 2 off the curve
    assert codec.decide_eip197(bytes(recs)) == 2
