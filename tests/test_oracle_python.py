"""The Python oracle: constants, group law, pairing, and the reference's own KATs (Poseidon)."""
import pytest

from conftest import load_golden, pt
from oracle import bn254 as b
from oracle import poseidon


def test_constants_from_bn_parameter():
    x = b.U
    assert b.P == 36 * x**4 + 36 * x**3 + 24 * x**2 + 6 * x + 1
    assert b.R == 36 * x**4 + 36 * x**3 + 18 * x**2 + 6 * x + 1
    assert b.P % 4 == 3
    # halo2curves' Montgomery one
    assert b.RP == 0x0e0a77c19a07df2f666ea36f7879462c0a78eb28f5c70b3dd35d438dc58f0d9d
    assert b.RR == 0x0e0a77c19a07df2f666ea36f7879462e36fc76959f60cd29ac96341c4ffffffb


def test_generators_on_curve_and_order_r():
    assert b.g1_on_curve(b.G1_GEN)
    assert b.g1_mul(b.G1_GEN, b.R) is None
    assert b.g2_on_curve(b.G2_GEN)
    assert b.g2_mul(b.G2_GEN, b.R) is None


def test_group_law():
    P1 = b.g1_mul(b.G1_GEN, 12345)
    P2 = b.g1_mul(b.G1_GEN, 678)
    assert b.g1_add(P1, P2) == b.g1_mul(b.G1_GEN, 12345 + 678)
    assert b.g1_add(P1, b.g1_neg(P1)) is None
    assert b.g1_add(P1, P1) == b.g1_mul(b.G1_GEN, 2 * 12345)
    assert b.g1_add(None, P1) == P1


def test_poseidon_mds_kat():
    kat = load_golden("poseidon_kat.json")
    _, mds = poseidon.spec(3, 8, 57)
    assert mds == [[int(v) for v in row] for row in kat["mds_t3"]]


@pytest.mark.parametrize("key", ["perm_x5_254_3", "perm_x5_254_5"])
def test_poseidon_permutation_kat(key):
    k = load_golden("poseidon_kat.json")[key]
    assert poseidon.permutation(k["input"], k["t"], k["r_f"], k["r_p"]) == [int(v) for v in k["output"]]


@pytest.mark.parametrize("key", ["perm_x5_254_3", "perm_x5_254_5"])
def test_poseidon_optimized_schedule_matches_kat_and_plain(key):
    """The reference's optimised schedule (OptimizedPoseidonSpec: folded constants, pre-sparse MDS,
    sparse partial-round matrices, poseidon.rs:170-328 / :469-500), restated in oracle/poseidon.py
    and compiled into the GPU kernel, reproduces the KAT and the plain HADES rounds."""
    import random
    k = load_golden("poseidon_kat.json")[key]
    t, rf, rp = k["t"], k["r_f"], k["r_p"]
    assert poseidon.permutation_optimized(k["input"], t, rf, rp) == [int(v) for v in k["output"]]
    rng = random.Random(t)
    for _ in range(4):
        st = [rng.randrange(poseidon.FR_MODULUS) for _ in range(t)]
        assert poseidon.permutation_optimized(st, t, rf, rp) == poseidon.permutation(st, t, rf, rp)
    sp = poseidon.optimized_spec(t, rf, rp)
    assert len(sp["sparse"]) == rp and len(sp["start"]) == rf // 2 + 1 and len(sp["end"]) == rf // 2 - 1


def test_pairing_tower_equals_generic_formulation():
    e = b.pairing(b.G1_GEN, b.G2_GEN)
    assert b.tower_to_poly(e) == b.pairing_generic(b.G1_GEN, b.G2_GEN)
    P1, Q1 = b.g1_mul(b.G1_GEN, 5), b.g2_mul(b.G2_GEN, 7)
    assert b.tower_to_poly(b.pairing(P1, Q1)) == b.pairing_generic(P1, Q1)


def test_pairing_bilinear_nondegenerate():
    e = b.pairing(b.G1_GEN, b.G2_GEN)
    assert e != b.F12_ONE
    assert b.f12_pow(e, b.R) == b.F12_ONE
    a, c = 31337, 4242
    assert b.pairing(b.g1_mul(b.G1_GEN, a), b.g2_mul(b.G2_GEN, c)) == b.f12_pow(e, a * c)


def test_final_exponentiation_chain_is_exact():
    f = b.multi_miller_loop([(b.G1_GEN, b.g2_prepare(b.G2_GEN))])
    easy = b.f12_mul(b.f12_conj(f), b.f12_inv(f))
    easy = b.f12_mul(b.f12_frob_n(easy, 2), easy)
    assert b.final_exp_hard_chain(easy) == b.f12_pow(easy, b.FINAL_EXP_HARD)


def test_decider_semantics():
    g2, sg2, accs = b.gen_decider_case(3, bad=[1])
    assert b.decide_all(g2, sg2, accs) == 1
    assert b.decide(g2, sg2, None, None)
    assert b.decide(g2, sg2, *accs[0])
    with pytest.raises(AssertionError):
        b.decide_all(g2, sg2, [])


def test_msm_restatements_agree_with_golden(golden_msm):
    for c in golden_msm["cases"]:
        if "scalars" not in c:
            continue
        sc = [int(s, 16) for s in c["scalars"]]
        bs = [pt(p) for p in c["bases"]]
        exp = pt(c["expected"])
        assert b.native_msm(sc, bs) == exp, c["name"]
        assert b.pippenger_msm(sc, bs) == exp, c["name"]


def test_generator_matches_golden(golden_msm):
    g = golden_msm["generator"]
    assert [hex(s) for s in b.gen_scalars(b.SEED_SCALARS, 8)] == g["scalars"]["values"]
    assert [[hex(p[0]), hex(p[1])] for p in b.gen_bases(b.SEED_BASES, 8)] == g["bases"]["values"]


def test_native_msm_empty_panics():
    with pytest.raises(ValueError, match="pairs should not be empty"):
        b.native_msm([], [])


def test_limb_codec_roundtrip():
    x = b.g1_mul(b.G1_GEN, 99)[0]
    limbs = b.fe_to_limbs(x)
    assert all(l < (1 << 88) for l in limbs)
    assert b.fe_from_limbs(limbs) == x


def test_poseidon_sponge_restatement_structure():
    """Sponge (poseidon.rs:412-467): padding and the exact-length extra permutation, checked by
    composing the KAT-pinned permutation by hand."""
    t, (rf, rp) = 3, poseidon.PARAMS[3]
    perm = lambda s: poseidon.permutation(s, t, rf, rp)  # noqa: E731
    s0 = [1 << 64, 0, 0]
    # empty buffer: one permutation of the padded empty chunk (state[1] += 1)
    sp = poseidon.Sponge(t)
    assert sp.squeeze() == perm([s0[0], 1, 0])[1]
    # one element: chunk [a] padded with 1 at state[2]; not exact -> no extra permutation
    sp = poseidon.Sponge(t)
    sp.update([5])
    assert sp.squeeze() == perm([s0[0], 5, 1])[1]
    # two elements (exact): full chunk, then the padded empty chunk
    sp = poseidon.Sponge(t)
    sp.update([5, 6])
    st = perm([s0[0], 5, 6])
    assert sp.squeeze() == perm([st[0], st[1] + 1, st[2]])[1]
    # inputs are reduced mod r like Fr
    a, c = poseidon.Sponge(t), poseidon.Sponge(t)
    a.update([3])
    c.update([3 + poseidon.FR_MODULUS])
    assert a.squeeze() == c.squeeze()


def test_codec_restatements_round_trip():
    pts = [b.g1_mul(b.G1_GEN, k) for k in (1, 2, 3, 12345, b.R - 1)] + [None]
    for p in pts:
        assert b.g1_decompress(b.g1_compress(p)) == p
        assert b.g1_evm_decode(b.g1_evm_encode(p)) == p
    with pytest.raises(b.CodecError):
        b.g1_evm_decode(b.P.to_bytes(32, "big") + (2).to_bytes(32, "big"))   # x >= p
    with pytest.raises(b.CodecError):
        b.g1_evm_decode((1).to_bytes(32, "big") + (3).to_bytes(32, "big"))   # off curve
    bad_x = next(x for x in range(1, 100) if b.sqrt_fp((x ** 3 + 3) % b.P) is None)
    with pytest.raises(b.CodecError):
        b.g1_decompress(bad_x.to_bytes(32, "little"))                        # no square root
    # limbs: SDK LIMBS = 3, BITS = 88
    lhs, rhs = b.g1_mul(b.G1_GEN, 77), b.g1_mul(b.G1_GEN, 99)
    limbs = sum((b.fe_to_limbs(c) for c in (lhs[0], lhs[1], rhs[0], rhs[1])), [])
    assert b.accumulator_from_limbs(limbs) == (lhs, rhs)
    with pytest.raises(b.CodecError):
        b.accumulator_from_limbs(limbs[:-1] + [limbs[-1] + 1])              # off curve
    with pytest.raises(b.CodecError):
        b.fe_from_limbs([0, 0, 1 << 100])                                    # > 2^256
    g2, sg2, accs = b.gen_decider_case(2)
    rec = b.eip197_input(g2, sg2, *accs[0])
    lhs2, g2p, rhs2, msg2 = b.eip197_parse(rec)
    assert (lhs2, g2p, rhs2, msg2) == (accs[0][0], g2, accs[0][1], b.g2_neg(sg2))
