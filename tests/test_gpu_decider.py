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
    g2, sg2, accs = b.gen_decider_case(16, seed=0xD3C1DE)
    accs = (accs * (n // 16))[:n]
    bad = 201
    accs[bad] = (b.g1_add(accs[bad][0], b.G1_GEN), accs[bad][1])
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
