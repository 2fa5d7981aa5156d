"""C++ CPU restatement (oracle/cpu/bn254_ref.cpp) against the golden fixtures."""
import numpy as np
import pytest

import os

from conftest import ROOT, pt, q2
from oracle import bn254 as b


def _pts(points):
    return np.frombuffer(b"".join(b.g1_bytes(p) for p in points), dtype=np.uint64).reshape(-1, 8).copy()


def _scs(scalars):
    return np.frombuffer(b"".join(int(s).to_bytes(32, "little") for s in scalars), dtype=np.uint64).reshape(-1, 4).copy()


def _to_pt(row):
    return b.g1_from_bytes(row.tobytes())


def test_generators_match_python(oracle_cpp, golden_msm):
    g = golden_msm["generator"]
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, 8)
    assert [hex(int.from_bytes(r.tobytes(), "little")) for r in S] == g["scalars"]["values"]
    B = oracle_cpp.gen_bases(b.SEED_BASES, 8)
    assert [[hex(p[0]), hex(p[1])] for p in map(_to_pt, B)] == g["bases"]["values"]
    B2 = oracle_cpp.gen_bases(b.SEED_BASES, 4, start=1000)
    assert [[hex(p[0]), hex(p[1])] for p in map(_to_pt, B2)] == g["bases_start_1000"]


def test_msm_golden(oracle_cpp, golden_msm):
    for c in golden_msm["cases"]:
        if "scalars" in c:
            S, B = _scs([int(s, 16) for s in c["scalars"]]), _pts([pt(p) for p in c["bases"]])
        else:
            S = oracle_cpp.gen_scalars(c["seeds"]["scalars"], c["n"])
            B = oracle_cpp.gen_bases(c["seeds"]["bases"], c["n"])
        exp = pt(c["expected"])
        assert _to_pt(oracle_cpp.msm_naive(B, S)) == exp, c["name"]
        for th in (1, 4):
            assert _to_pt(oracle_cpp.msm_pippenger(B, S, th)) == exp, (c["name"], th)


def test_decider_golden(oracle_cpp, golden_decider):
    for c in golden_decider["cases"]:
        g2 = np.frombuffer(b.g2_bytes(q2(c["g2"])), dtype=np.uint64)
        sg2 = np.frombuffer(b.g2_bytes(q2(c["s_g2"])), dtype=np.uint64)
        L, R = _pts([pt(p) for p in c["lhs"]]), _pts([pt(p) for p in c["rhs"]])
        ff, gt = oracle_cpp.decide_all(g2, sg2, L, R, threads=2, want_gt=True)
        assert ff == c["first_fail"], c["name"]
        if "gt" in c:
            got = [[hex(int.from_bytes(gt[i][4 * k:4 * k + 4].tobytes(), "little")) for k in range(12)]
                   for i in range(len(c["lhs"]))]
            assert got == c["gt"]


def test_accumulate_golden(oracle_cpp, golden_decider):
    a = golden_decider["accumulate"]
    L, R = _pts([pt(p) for p in a["lhs"]]), _pts([pt(p) for p in a["rhs"]])
    r = np.frombuffer(int(a["r"], 16).to_bytes(32, "little"), dtype=np.uint64)
    ol, orr = oracle_cpp.accumulate(L, R, r)
    assert [_to_pt(ol), _to_pt(orr)] == [pt(a["expected"][0]), pt(a["expected"][1])]


def test_empty_inputs_panic(oracle_cpp):
    with pytest.raises(AssertionError, match="pairs should not be empty"):
        oracle_cpp.msm_naive(np.zeros((0, 8), np.uint64), np.zeros((0, 4), np.uint64))


def test_decide_fpmul_count_is_the_bench_constant():
    """bench.py's FPMUL_RESTATEMENT is the instrumented restatement's Fq-product count per decide."""
    import re
    from oracle import cpu_ref
    from svgpu import encoding as enc
    g2, sg2, accs = b.gen_decider_case(2)
    L = enc.bases_array([a[0] for a in accs])
    R = enc.bases_array([a[1] for a in accs])
    cnt = cpu_ref.count_decide_fpmul(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64),
                                     L[0], R[0])
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert int(re.search(r"FPMUL_RESTATEMENT = (\d+)", src).group(1)) == cnt


def test_decide_fpmul_h2c_count_is_the_bench_denominator_and_gt_agrees(oracle_cpp):
    """bench.py's FPMUL_H2C_COUNTED (the decider roofline's work unit) is the Fq-product count of the
    halo2curves-structured restatement (bn254_ref.cpp namespace h2c: cyclotomic squarings, sparse
    034 lines, exp_by_x, Scott et al. hard part), and that restatement's Gt value equals the plain
    restatement's for accepted and rejected accumulators alike (decider.rs:60-68)."""
    import re
    from oracle import cpu_ref
    from svgpu import encoding as enc
    g2, sg2, accs = b.gen_decider_case(3, bad=[1])
    G2, SG2 = np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64)
    L = enc.bases_array([a[0] for a in accs])
    R = enc.bases_array([a[1] for a in accs])
    ff, gts = oracle_cpp.decide_all(G2, SG2, L, R, threads=1, want_gt=True)
    assert ff == 1
    counts = set()
    for i in range(3):
        cnt, gt = cpu_ref.count_decide_fpmul_h2c(G2, SG2, L[i], R[i])
        counts.add(cnt)
        assert (gt == gts[i]).all()
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert counts == {int(re.search(r"FPMUL_H2C_COUNTED = (\d+)", src).group(1))}


def test_h2c_line_prep_count_is_the_bench_constant():
    """bench.py's FPMUL_H2C_LINE_PREP: the Fq products of the two G2 line preparations inside one
    h2c decide (G2Prepared::from, decider.rs:64), which the GPU decider caches per deciding key; the
    roofline's frac_without_line_prep drops them."""
    import re
    from oracle import cpu_ref
    g2, sg2, _ = b.gen_decider_case(2)
    cnt = cpu_ref.count_h2c_prepare(np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64))
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert int(re.search(r"FPMUL_H2C_LINE_PREP = (\d+)", src).group(1)) == cnt
    assert cnt < int(re.search(r"FPMUL_H2C_COUNTED = (\d+)", src).group(1))
