"""GPU KZG decider + accumulation parity through the C ABI against the oracles."""
import numpy as np
import pytest
import torch

from conftest import pt, q2
from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def _dev(points, device):
    from svgpu import encoding as enc
    return torch.from_numpy(enc.bases_array(points).view(np.int64)).to(device)


def test_golden_first_fail_and_gt(gpu, golden_decider):
    import svgpu
    from svgpu import device as dv
    for c in golden_decider["cases"]:
        lhs = [pt(p) for p in c["lhs"]]
        rhs = [pt(p) for p in c["rhs"]]
        ff, verdicts, gts = dv.decide(q2(c["g2"]), q2(c["s_g2"]), _dev(lhs, gpu), _dev(rhs, gpu),
                                      svgpu.SV_CANONICAL, want_gt=True)
        assert ff == c["first_fail"], c["name"]
        if "gt" in c:
            assert [[hex(v) for v in g] for g in gts] == c["gt"]
        # host API + reference-shaped mirror
        dk = svgpu.KzgDecidingKey(b.G1_GEN, q2(c["g2"]), q2(c["s_g2"]))
        accs = [svgpu.KzgAccumulator(l, r) for l, r in zip(lhs, rhs)]
        assert svgpu.KzgAs.first_failure(dk, accs) == c["first_fail"]
        if c["first_fail"] >= 0:
            with pytest.raises(svgpu.AssertionFailure, match=r"e\(lhs, g2\)·e\(rhs, -s_g2\) == O"):
                svgpu.KzgAs.decide_all(dk, accs)
        else:
            svgpu.KzgAs.decide_all(dk, accs)


def test_pairing_value_e_g1_g2(gpu, golden_decider):
    """e(G1, G2) through the decider: lhs = G1, rhs = identity -> Gt = e(G1, g2)."""
    from svgpu import device as dv
    ff, _, gts = dv.decide(b.G2_GEN, b.G2_GEN, _dev([b.G1_GEN], gpu), _dev([None], gpu), want_gt=True)
    assert ff == 0
    assert [hex(v) for v in gts[0]] == golden_decider["pairing"]["e_g1_g2"]


def test_256_accumulators_vs_cpp(gpu, oracle_cpp):
    import svgpu
    from svgpu import encoding as enc
    n = 256
    bad = 201
    g2, sg2, accs = b.gen_decider_case(n, seed=0xD3C1DE, bad=[bad])  # 256 distinct accumulators
    L = enc.bases_array([a[0] for a in accs])
    R = enc.bases_array([a[1] for a in accs])
    dk = svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2)
    from svgpu.kzg import decide_arrays
    got = decide_arrays(dk, L, R)
    exp, _ = oracle_cpp.decide_all(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64),
                                   L, R, threads=0)
    assert got == exp == bad


def test_montgomery_form_decider(gpu):
    import svgpu
    from svgpu import encoding as enc
    from svgpu.kzg import decide_arrays
    g2, sg2, accs = b.gen_decider_case(5, bad=[4])
    dk = svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2)
    L = enc.bases_array([a[0] for a in accs], svgpu.SV_MONTGOMERY)
    R = enc.bases_array([a[1] for a in accs], svgpu.SV_MONTGOMERY)
    assert decide_arrays(dk, L, R, svgpu.SV_MONTGOMERY) == 4


def test_accumulate_golden_and_decide(gpu, golden_decider):
    import svgpu
    a = golden_decider["accumulate"]
    accs = [svgpu.KzgAccumulator(pt(l), pt(r)) for l, r in zip(a["lhs"], a["rhs"])]
    out = svgpu.KzgAs.create_proof(accs, int(a["r"], 16))
    assert [out.lhs, out.rhs] == [pt(a["expected"][0]), pt(a["expected"][1])]
    # an int-like r (numbers.Integral, e.g. a numpy integer) is r too, not a transcript
    small = svgpu.KzgAs.create_proof(accs, np.uint64(12345))
    assert (small.lhs, small.rhs) == b.accumulate([(pt(l), pt(r)) for l, r in zip(a["lhs"], a["rhs"])], 12345)


def test_aggregation_64_end_to_end(gpu):
    """Config 5 restated: 64 valid accumulators -> accumulate (2 x 64-term MSM) -> one decide."""
    import svgpu
    g2, sg2, accs = b.gen_decider_case(64, seed=0x64)
    dk = svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2)
    r = b.gen_scalar(0x7777, 0)
    acc = svgpu.KzgAs.create_proof([svgpu.KzgAccumulator(*x) for x in accs], r)
    assert (acc.lhs, acc.rhs) == b.accumulate(accs, r)
    svgpu.KzgAs.decide(dk, acc)
    bad = svgpu.KzgAccumulator(b.g1_add(acc.lhs, b.G1_GEN), acc.rhs)
    with pytest.raises(svgpu.AssertionFailure):
        svgpu.KzgAs.decide(dk, bad)


@pytest.mark.parametrize("lanes", ["256", "48", "24", "auto"])
def test_both_decider_kernels_gt_and_first_fail(gpu, oracle_cpp, monkeypatch, lanes):
    """k_decide_wg (one 4-wave block per accumulator) and k_decide_lanes (one wave per accumulator)
    give the oracle's Gt values and first failure; 'auto' with more accumulators than CUs takes
    the single-wave kernel for the whole batch."""
    import svgpu
    from svgpu import device as dv
    from svgpu import encoding as enc
    if lanes != "auto":
        monkeypatch.setenv("SVGPU_DECIDER_LANES", lanes)
    n = 300 if lanes == "auto" else 40
    g2, sg2, accs = b.gen_decider_case(20, seed=0xBEEF, bad=[13])
    accs = (accs * (n // 20 + 1))[:n]
    accs[n - 3] = (None, None)                                  # identity pair: passes
    L, R = enc.bases_array([a[0] for a in accs]), enc.bases_array([a[1] for a in accs])
    ff, verdicts, gts = dv.decide(g2, sg2, _dev([a[0] for a in accs], gpu), _dev([a[1] for a in accs], gpu),
                                  svgpu.SV_CANONICAL, want_gt=True)
    eff, egt = oracle_cpp.decide_all(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64),
                                     L, R, threads=0, want_gt=True)
    assert ff == eff == 13
    assert sum(1 for v in verdicts if not v) == n // 20 + (1 if n % 20 > 13 else 0)
    for i in (0, 13, n - 3, n - 1):
        assert [int(x) for x in gts[i]] == [enc.limbs_to_int(egt[i][4 * c:4 * c + 4]) for c in range(12)], i


def test_create_proof_transcript_golden(gpu, golden_decider):
    """KzgAs::create_proof(instances, transcript) with a fresh Poseidon transcript
    (accumulation.rs:146-195): r squeezed after absorbing every lhs_i, rhs_i (common_ec_point,
    transcript/halo2.rs:214-226) equals the oracle's, and so do the two r^i MSMs."""
    import svgpu
    c = golden_decider["create_proof"]
    accs = [svgpu.KzgAccumulator(pt(l), pt(r)) for l, r in zip(c["lhs"], c["rhs"])]
    out = svgpu.KzgAs.create_proof(accs, svgpu.PoseidonTranscript())
    assert svgpu.KzgAs.last_challenge == int(c["r"], 16)
    assert [out.lhs, out.rhs] == [pt(c["expected"][0]), pt(c["expected"][1])]


def test_config5_create_proof_64_transcript_vs_oracle(gpu):
    """Config 5: 64 accumulators -> transcript-derived r -> accumulate -> decide, against the oracle;
    also in Montgomery form through the C ABI (r and the outputs as Montgomery limbs)."""
    import ctypes
    import svgpu
    from svgpu import _lib, encoding as enc
    g2, sg2, accs = b.gen_decider_case(64, seed=0x64)
    (el, er), r, state = b.create_proof(accs)
    inst = [svgpu.KzgAccumulator(*x) for x in accs]
    out = svgpu.KzgAs.create_proof(inst)
    assert svgpu.KzgAs.last_challenge == r
    assert (out.lhs, out.rhs) == (el, er)
    svgpu.KzgAs.decide(svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2), out)
    # Montgomery form, with the sponge state handed back
    M = svgpu.SV_MONTGOMERY
    L = enc.bases_array([a[0] for a in accs], M)
    R_ = enc.bases_array([a[1] for a in accs], M)
    ol, orr = _lib.sv_g1_affine(), _lib.sv_g1_affine()
    rr = np.zeros(4, np.uint64)
    st = enc.ints_to_limbs([(1 << 64) * (1 << 256) % enc.R, 0, 0])  # fresh state, Montgomery
    _lib.check(_lib.lib.sv_bn254_kzg_create_proof(L.ctypes.data, R_.ctypes.data, 64, M, 0, ctypes.byref(ol),
                                                  ctypes.byref(orr), st.ctypes.data, rr.ctypes.data), "create_proof")
    mont = lambda v: v * (1 << 256) % enc.R  # noqa: E731
    assert enc.limbs_to_int(rr) == mont(r)
    assert [enc.limbs_to_int(row) for row in st] == [mont(v) for v in state]
    assert (enc.g1_from_struct(ol, M), enc.g1_from_struct(orr, M)) == (el, er)


def test_create_proof_continues_a_used_transcript(gpu):
    """A transcript squeezed before (empty buffer): its sponge state goes into the library call and
    the state after the squeeze comes back, as the reference's transcript would hold it."""
    import svgpu
    g2, sg2, accs = b.gen_decider_case(5, seed=0x55)
    tr = svgpu.PoseidonTranscript()
    tr.common_scalar(12345)
    c0 = tr.squeeze_challenge()
    state0 = list(tr.buf.state)
    out = svgpu.KzgAs.create_proof([svgpu.KzgAccumulator(*x) for x in accs], tr)
    (el, er), r, state = b.create_proof(accs, state0)
    assert c0 != r and svgpu.KzgAs.last_challenge == r
    assert (out.lhs, out.rhs) == (el, er)
    assert tr.buf.state == state
    # a transcript with buffered input is absorbed and squeezed through svgpu.poseidon (device sponge)
    tr2 = svgpu.PoseidonTranscript()
    tr2.common_scalar(7)
    out2 = svgpu.KzgAs.create_proof([svgpu.KzgAccumulator(*x) for x in accs], tr2)
    from oracle import poseidon as op
    sp = op.Sponge(3)
    sp.update([7])
    for a in accs:
        op.transcript_common_ec_point(sp, a[0])
        op.transcript_common_ec_point(sp, a[1])
    r2 = sp.squeeze()
    assert (out2.lhs, out2.rhs) == b.accumulate(accs, r2)


def test_create_proof_rejects_identity_and_empty(gpu):
    import svgpu
    from svgpu.loader import ReferencePanic
    g2, sg2, accs = b.gen_decider_case(3, seed=0x33)
    inst = [svgpu.KzgAccumulator(*x) for x in accs] + [svgpu.KzgAccumulator(None, accs[0][1])]
    with pytest.raises(svgpu.ArgumentError, match="Invalid elliptic curve point encoding"):
        svgpu.KzgAs.create_proof(inst)
    with pytest.raises(ReferencePanic):
        svgpu.KzgAs.create_proof([])


def test_gt_equals_halo2curves_structured_restatement(gpu, oracle_cpp):
    """The kernel's Gt value equals the one of the C++ restatement that follows halo2curves'
    structure (bn254_ref.cpp namespace h2c: complex / Granger-Scott cyclotomic squarings, sparse
    034 lines, exp_by_x and the Scott et al. hard-part chain) -- accepted and rejected accumulators
    alike (decider.rs:60-68; the reference's final_exponentiation, external)."""
    from oracle import cpu_ref
    from svgpu import device as dv, encoding as enc
    g2, sg2, accs = b.gen_decider_case(4, seed=0x6767, bad=[1, 3])
    ff, _, gts = dv.decide(g2, sg2, _dev([a[0] for a in accs], gpu), _dev([a[1] for a in accs], gpu), want_gt=True)
    assert ff == 1
    G2, SG2 = np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64)
    L = enc.bases_array([a[0] for a in accs])
    R = enc.bases_array([a[1] for a in accs])
    for i in range(4):
        _, gt = cpu_ref.count_decide_fpmul_h2c(G2, SG2, L[i], R[i])
        limbs = [sum(int(gt[8 * c + 4 * h + j]) << (64 * j) for j in range(4)) for c in range(6) for h in range(2)]
        assert gts[i] == limbs, i


@pytest.mark.parametrize("env", ["SVGPU_DECIDER_WIDE=0", "SVGPU_DECIDER_PAIR=0", "SVGPU_DECIDER_KC=0",
                                 "SVGPU_DECIDER_WIDE=0 SVGPU_DECIDER_PAIR=0"])
def test_decider_prologue_variants(gpu, oracle_cpp, monkeypatch, env):
    """k_decide_wg's prologue options (the round-5 one-term-per-lane products and their round-4
    form, paired Miller steps, pair products from the key's constants) all give the oracle's Gt
    values, verdicts and first failure -- identity points included."""
    import svgpu
    from svgpu import device as dv
    from svgpu import encoding as enc
    for kv in env.split():
        k, v = kv.split("=")
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SVGPU_DECIDER_LANES", "256")
    n = 12
    g2, sg2, accs = b.gen_decider_case(n, seed=0xC0DE, bad=[7])
    accs[4] = (None, None)                                      # identity pair: passes
    accs[9] = (accs[9][0], None)                                # rhs identity: e(lhs, g2) != 1
    L, R = enc.bases_array([a[0] for a in accs]), enc.bases_array([a[1] for a in accs])
    ff, verdicts, gts = dv.decide(g2, sg2, _dev([a[0] for a in accs], gpu), _dev([a[1] for a in accs], gpu),
                                  svgpu.SV_CANONICAL, want_gt=True)
    eff, egt = oracle_cpp.decide_all(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64),
                                     L, R, threads=0, want_gt=True)
    assert ff == eff == 7
    for i in range(n):
        assert [int(x) for x in gts[i]] == [enc.limbs_to_int(egt[i][4 * c:4 * c + 4]) for c in range(12)], i


def test_decider_verdict_copy_path(gpu, oracle_cpp, monkeypatch):
    """SVGPU_DECIDE_ZC=0: verdicts through a device buffer and a copy (the default writes them
    straight into pinned host memory) -- same first failure and verdicts."""
    import svgpu
    from svgpu import device as dv
    from svgpu import encoding as enc
    g2, sg2, accs = b.gen_decider_case(10, seed=0xD1CE, bad=[3, 8])
    L, R = enc.bases_array([a[0] for a in accs]), enc.bases_array([a[1] for a in accs])
    got = {}
    for zc in ("1", "0"):
        monkeypatch.setenv("SVGPU_DECIDE_ZC", zc)
        ff, verdicts, _ = dv.decide(g2, sg2, _dev([a[0] for a in accs], gpu), _dev([a[1] for a in accs], gpu),
                                    svgpu.SV_CANONICAL)
        got[zc] = (ff, verdicts)
    eff, _ = oracle_cpp.decide_all(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64),
                                   L, R, threads=0, want_gt=False)
    assert got["1"] == got["0"] and got["1"][0] == eff == 3
    assert [i for i, v in enumerate(got["1"][1]) if not v] == [3, 8]


@pytest.mark.parametrize("n,small_off", [(257, False), (1000, False), (64, True), (5, True)])
def test_accumulate_pipeline_route_vs_cpp(gpu, oracle_cpp, monkeypatch, n, small_off):
    """sv_bn254_kzg_accumulate on the single-MSM pipeline route -- more accumulators than the
    small-MSM window path takes (n > 256), or that path switched off (SVGPU_SMALL_MSM=0) -- against
    the C++ oracle's r^i MSMs (accumulation.rs:177-192, loader.rs:71-78).  Regression for ADVICE r05
    (high): the route had lost its input uploads and the r^i powers."""
    import ctypes
    import svgpu
    from svgpu import _lib, encoding as enc
    if small_off:
        monkeypatch.setenv("SVGPU_SMALL_MSM", "0")
    L = oracle_cpp.gen_bases(0xACC0 + n, n)
    R_ = oracle_cpp.gen_bases(0xACC1 + n, n)
    r = b.gen_scalar(0xACC2, n)
    el, er = oracle_cpp.accumulate(L, R_, enc.ints_to_limbs([r])[0])
    # twice: the second call reuses a pooled workspace that still holds the first call's data
    for rr in (r, (r * 3 + 1) % b.R):
        ol, orr = _lib.sv_g1_affine(), _lib.sv_g1_affine()
        _lib.check(_lib.lib.sv_bn254_kzg_accumulate(L.ctypes.data, R_.ctypes.data, n, ctypes.byref(enc.fe_struct(rr)),
                                                    svgpu.SV_CANONICAL, 0, ctypes.byref(ol), ctypes.byref(orr)),
                   "sv_bn254_kzg_accumulate")
        if rr == r:
            assert enc.g1_from_struct(ol) == enc.g1_from_limbs(el)
            assert enc.g1_from_struct(orr) == enc.g1_from_limbs(er)
        else:
            e2l, e2r = oracle_cpp.accumulate(L, R_, enc.ints_to_limbs([rr])[0])
            assert (enc.g1_from_struct(ol), enc.g1_from_struct(orr)) == (enc.g1_from_limbs(e2l), enc.g1_from_limbs(e2r))


def test_create_proof_300_accumulators_vs_oracle(gpu, oracle_cpp):
    """create_proof over 300 accumulators (the pipeline route for its r^i MSMs): r from the
    transcript restatement, the MSMs from the C++ oracle."""
    import svgpu
    from oracle import poseidon as op
    from svgpu import encoding as enc
    n = 300
    L = oracle_cpp.gen_bases(0xC300, n)
    R_ = oracle_cpp.gen_bases(0xC301, n)
    accs = [(enc.g1_from_limbs(L[i]), enc.g1_from_limbs(R_[i])) for i in range(n)]
    sp = op.Sponge(3)
    for a in accs:
        op.transcript_common_ec_point(sp, a[0])
        op.transcript_common_ec_point(sp, a[1])
    r = sp.squeeze()
    out = svgpu.KzgAs.create_proof([svgpu.KzgAccumulator(*a) for a in accs])
    assert svgpu.KzgAs.last_challenge == r
    el, er = oracle_cpp.accumulate(L, R_, enc.ints_to_limbs([r])[0])
    assert (out.lhs, out.rhs) == (enc.g1_from_limbs(el), enc.g1_from_limbs(er))
