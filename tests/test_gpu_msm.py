"""GPU MSM parity through the C ABI (libsvgpu's HIP kernels) against the oracles."""
import numpy as np
import pytest
import torch

from conftest import pt
from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def _to_pt(row):
    return b.g1_from_bytes(np.asarray(row, dtype=np.uint64).tobytes())


def _golden_inputs(c, oracle_cpp):
    from svgpu import encoding as enc
    if "scalars" in c:
        return enc.bases_array([pt(p) for p in c["bases"]]), enc.scalars_array([int(s, 16) for s in c["scalars"]])
    return (oracle_cpp.gen_bases(c["seeds"]["bases"], c["n"]), oracle_cpp.gen_scalars(c["seeds"]["scalars"], c["n"]))


def test_golden_host_api_both_forms(gpu, golden_msm, oracle_cpp):
    import svgpu
    from svgpu import encoding as enc
    for c in golden_msm["cases"]:
        B, S = _golden_inputs(c, oracle_cpp)
        exp = pt(c["expected"])
        assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp, c["name"]
        pts = [enc.g1_from_limbs(r) for r in B]
        sc = [enc.limbs_to_int(r) for r in S]
        Bm, Sm = enc.bases_array(pts, svgpu.SV_MONTGOMERY), enc.scalars_array(sc, svgpu.SV_MONTGOMERY)
        assert svgpu.msm_arrays(Bm, Sm, svgpu.SV_MONTGOMERY) == exp, c["name"]


def test_native_loader_mirror(gpu, golden_msm):
    import svgpu
    c = next(c for c in golden_msm["cases"] if c["name"] == "mixed_edges")
    pairs = [(int(s, 16), pt(p)) for s, p in zip(c["scalars"], c["bases"])]
    assert svgpu.NativeLoader.multi_scalar_multiplication(pairs) == pt(c["expected"])


def test_device_generators_match_oracle(gpu, oracle_cpp):
    import svgpu
    from svgpu import device as dv
    n = 5000
    for form in (svgpu.SV_CANONICAL, svgpu.SV_MONTGOMERY):
        Bd = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 123, form)
        Sd = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 123, form)
        torch.cuda.synchronize()
        Bh = Bd.cpu().numpy().view(np.uint64)
        Sh = Sd.cpu().numpy().view(np.uint64)
        Bo = oracle_cpp.gen_bases(b.SEED_BASES, n, start=123)
        So = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=123)
        if form == svgpu.SV_MONTGOMERY:
            from svgpu import encoding as enc
            Bh = enc.bases_array([enc.g1_from_limbs(r, form) for r in Bh])
            Sh = enc.scalars_array([enc._from_form(enc.limbs_to_int(r), b.R, form) for r in Sh])
        assert (Bh == Bo).all() and (Sh == So).all()


@pytest.mark.parametrize("n", [1, 2, 5, 63, 64, 65, 1000, 4095, 4096, 65537])
def test_random_sizes_vs_cpp_pippenger(gpu, oracle_cpp, n):
    from svgpu import device as dv
    import svgpu
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=7 * n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=7 * n)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    Bd = torch.from_numpy(B.view(np.int64)).to(gpu)
    Sd = torch.from_numpy(S.view(np.int64)).to(gpu)
    assert dv.msm(Bd, Sd, svgpu.SV_CANONICAL) == exp


@pytest.mark.parametrize("bits", ["", "10"])
@pytest.mark.parametrize("halves", ["0", "1"])
@pytest.mark.parametrize("glv", ["0", "1"])
def test_sort_stored_halves(gpu, oracle_cpp, monkeypatch, halves, glv, bits):
    """The device path's scatter pass reading the digits source the histogram pass stored (GLV
    halves with their signs, or the canonical scalar) against recomputing it, both input forms
    (Montgomery scalars are converted by the histogram pass), with edge scalars mixed in, at the
    default window and at 10-bit windows (256-point sort blocks)."""
    from svgpu import device as dv
    from svgpu import encoding as enc
    import svgpu
    monkeypatch.setenv("SVGPU_SORT_HALVES", halves)
    monkeypatch.setenv("SVGPU_GLV", glv)
    if bits:  # more windows: 256-point sort blocks once a point has more than 20 entries
        monkeypatch.setenv("SVGPU_WINDOW_BITS", bits)
    n = 40000
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=5 * n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=5 * n)
    edge = [0, 1, 2, b.R - 1, b.R - 2, (b.R - 1) // 2, 1 << 127, (1 << 127) - 1, 1 << 128, b.R >> 1]
    S[:len(edge)] = enc.scalars_array(edge)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    Bd = torch.from_numpy(B.view(np.int64)).to(gpu)
    Sd = torch.from_numpy(S.view(np.int64)).to(gpu)
    assert dv.msm(Bd, Sd, svgpu.SV_CANONICAL) == exp
    Sm = enc.scalars_array([enc.limbs_to_int(r) for r in S], svgpu.SV_MONTGOMERY)
    Bm = enc.bases_array([enc.g1_from_limbs(r) for r in B], svgpu.SV_MONTGOMERY)
    assert dv.msm(torch.from_numpy(Bm.view(np.int64)).to(gpu), torch.from_numpy(Sm.view(np.int64)).to(gpu),
                  svgpu.SV_MONTGOMERY) == exp


@pytest.mark.parametrize("pf", ["0", "1"])
def test_hist_prefetch(gpu, oracle_cpp, monkeypatch, pf):
    """The histogram pass with the next point's loads one iteration ahead (round 6, the 29-bit table
    path) against the plain loop: a ragged size (the last block partial, threads whose next point
    is past the end), both input forms, and invalid Montgomery inputs still flagged (a scalar not
    below r, a base coordinate not below p) from inside the prefetching loop."""
    from svgpu import device as dv
    from svgpu import encoding as enc
    import svgpu
    monkeypatch.setenv("SVGPU_HIST_PF", pf)
    n = 40001
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=7 * n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=7 * n)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert dv.msm(torch.from_numpy(B.view(np.int64)).to(gpu), torch.from_numpy(S.view(np.int64)).to(gpu),
                  svgpu.SV_CANONICAL) == exp
    Sm = enc.scalars_array([enc.limbs_to_int(r) for r in S], svgpu.SV_MONTGOMERY)
    Bm = enc.bases_array([enc.g1_from_limbs(r) for r in B], svgpu.SV_MONTGOMERY)
    assert dv.msm(torch.from_numpy(Bm.view(np.int64)).to(gpu), torch.from_numpy(Sm.view(np.int64)).to(gpu),
                  svgpu.SV_MONTGOMERY) == exp
    bad_s = Sm.copy()
    bad_s[n - 1] = enc.ints_to_limbs([b.R])[0]  # the last point: reached through the prefetch
    with pytest.raises(svgpu.ArgumentError):
        dv.msm(torch.from_numpy(Bm.view(np.int64)).to(gpu), torch.from_numpy(bad_s.view(np.int64)).to(gpu),
               svgpu.SV_MONTGOMERY)
    bad_b = Bm.copy()
    bad_b[n - 1][:4] = enc.ints_to_limbs([b.P])[0]  # x = p: not reduced
    with pytest.raises(svgpu.ArgumentError):
        dv.msm(torch.from_numpy(bad_b.view(np.int64)).to(gpu), torch.from_numpy(Sm.view(np.int64)).to(gpu),
               svgpu.SV_MONTGOMERY)


def test_adversarial_single_bucket(gpu, oracle_cpp):
    """All scalars equal: every window's digits land in ONE bucket (maximal bucket skew)."""
    import svgpu
    n = 20000
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = np.tile(np.array([0xDEADBEEFCAFEBABE, 0x1234, 0, 0x0FFF], np.uint64), (n, 1))
    assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0))


def test_repeated_and_cancelling_points(gpu, oracle_cpp):
    import svgpu
    n = 3000
    B = oracle_cpp.gen_bases(b.SEED_BASES, 10)
    B = np.concatenate([B] * (n // 10))
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, 10)
    S = np.concatenate([S] * (n // 10))
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S) == exp
    # P and -P with equal scalars cancel to the identity
    from svgpu import encoding as enc
    pts = [enc.g1_from_limbs(r) for r in B[:10]]
    negs = [b.g1_neg(p) for p in pts]
    allp = enc.bases_array(pts + negs)
    sc = np.concatenate([S[:10], S[:10]])
    assert svgpu.msm_arrays(allp, sc) is None


def test_invalid_scalar_rejected(gpu):
    import svgpu
    from svgpu import encoding as enc
    B = enc.bases_array([b.G1_GEN])
    S = enc.ints_to_limbs([b.R])
    with pytest.raises(svgpu.ArgumentError):
        svgpu.msm_arrays(B, S)


def test_full_size_2_20_parity_and_properties(gpu, oracle_cpp):
    """Config 2 size: GPU == C++ Pippenger at 2^20; linearity and shard-additivity properties."""
    import svgpu
    from svgpu import device as dv, encoding as enc
    n = 1 << 20
    Bd = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 0, svgpu.SV_MONTGOMERY)
    Sd = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_MONTGOMERY)
    got = dv.msm(Bd, Sd, svgpu.SV_MONTGOMERY)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    assert got == _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    # shard additivity: two halves folded == whole
    h = n // 2
    p1 = dv.msm_partial(Bd[:h], Sd[:h], svgpu.SV_MONTGOMERY)
    p2 = dv.msm_partial(Bd[h:], Sd[h:], svgpu.SV_MONTGOMERY)
    assert svgpu.fold_partials([p1, p2]) == got
    # linearity in the scalars: MSM(2 s) == 2 MSM(s) (scalars doubled mod r on the host)
    S2 = enc.scalars_array([(2 * enc.limbs_to_int(r)) % b.R for r in S[:4096]])
    g1 = svgpu.msm_arrays(B[:4096], S[:4096])
    g2 = svgpu.msm_arrays(B[:4096], S2)
    assert g2 == b.g1_add(g1, g1)


def test_multi_device_host_api_consistent(gpu, oracle_cpp):
    import svgpu
    n = 10000
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    for g in (0, 1, 2):
        assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL, num_gpus=g) == exp


def test_adversarial_all_equal_scalars_2_18_is_fast(gpu, oracle_cpp):
    """Every window's 2^18 entries land in ONE bucket: the heavy-bucket fixup path must keep this
    both exact and fast (a serial join of 2^13 pieces per window took ~0.1 s before)."""
    import time
    import svgpu
    from svgpu import device as dv
    n = 1 << 18
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = np.tile(np.array([0x0123456789ABCDEF, 0xFEDCBA9876543210, 0x1111111111111111, 0x0222222222222222],
                         np.uint64), (n, 1))
    Bd = torch.from_numpy(B.view(np.int64)).to(gpu)
    Sd = torch.from_numpy(S.view(np.int64)).to(gpu)
    got = dv.msm(Bd, Sd, svgpu.SV_CANONICAL)
    t0 = time.perf_counter()
    dv.msm(Bd, Sd, svgpu.SV_CANONICAL)
    dt = time.perf_counter() - t0
    assert got == _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert dt < 0.05, f"skewed-bucket MSM took {dt * 1e3:.1f} ms"


@pytest.mark.parametrize("bits", [4, 5, 9, 13, 14, 15, 16])
def test_window_bits_override(gpu, oracle_cpp, bits, monkeypatch):
    """Every window size (incl. short top windows that concentrate digits) gives the same point."""
    import svgpu
    monkeypatch.setenv("SVGPU_WINDOW_BITS", str(bits))
    n = 20000
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=99)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=99)
    assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0))


@pytest.mark.parametrize("glv", ["0", "1"])
def test_edge_scalars(gpu, oracle_cpp, glv, monkeypatch):
    """Scalars at window and GLV-decomposition edges (k = lambda gives k1 = 0, k2 = 1; multiples and
    neighbours of lambda, of r, of 2^127 / 2^128) against the reference Pippenger restatement, with
    the single-MSM pipeline's GLV split forced off and on (SVGPU_GLV)."""
    import random
    import svgpu
    monkeypatch.setenv("SVGPU_GLV", glv)
    from svgpu import encoding as enc
    lam = 0xB3C4D79D41A917585BFC41088D8DAAA78B17EA66B99C90DD
    r = b.R
    ks = [0, 1, 2, lam, lam + 1, lam - 1, r - lam, (lam * lam) % r, r - 1, r - 2, (r - 1) // 2, (r + 1) // 2,
          1 << 126, (1 << 127) - 1, 1 << 127, 1 << 128, (1 << 128) + lam, (2 * lam) % r, (3 * lam) % r]
    ks += [(t * ((1 << 127) - 1) + lam * t) % r for t in range(1, 40)]
    rng = random.Random(5)
    ks += [rng.randrange(r) for _ in range(200)]
    n = len(ks)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=7)
    S = enc.scalars_array(ks)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp
    # each edge scalar alone (single-term MSMs) -- the split of every k is exercised in isolation
    for k in ks[:19]:
        Sk = enc.scalars_array([k])
        assert svgpu.msm_arrays(B[:1], Sk) == _to_pt(oracle_cpp.msm_pippenger(B[:1], Sk, 0)), hex(k)


@pytest.mark.parametrize("glv", ["0", "1"])
@pytest.mark.parametrize("n", [2, 3, 65, 4097, 20000, 65537])
def test_glv_split_on_off(gpu, oracle_cpp, n, glv, monkeypatch):
    """The single-MSM pipeline with and without the GLV split (2n virtual points, 128-bit halves,
    phi(P) table) gives the reference Pippenger's point, both input forms."""
    import svgpu
    from svgpu import encoding as enc
    monkeypatch.setenv("SVGPU_GLV", glv)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=31 * n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=31 * n)
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp
    if n <= 4097:
        pts = [enc.g1_from_limbs(r) for r in B]
        sc = [enc.limbs_to_int(r) for r in S]
        Bm = enc.bases_array(pts, svgpu.SV_MONTGOMERY)
        Sm = enc.scalars_array(sc, svgpu.SV_MONTGOMERY)
        assert svgpu.msm_arrays(Bm, Sm, svgpu.SV_MONTGOMERY) == exp


@pytest.mark.parametrize("phi64", ["0", "1"])
@pytest.mark.parametrize("n", [3, 4097, 65537])
def test_glv_phi_table_layouts(gpu, oracle_cpp, n, phi64, monkeypatch):
    """GLV with the beta-x-only table (k2 entries read y from the bases) and with whole phi(P)
    records (SVGPU_GLV_PHI64), identity bases included, against the reference Pippenger."""
    import svgpu
    monkeypatch.setenv("SVGPU_GLV", "1")
    monkeypatch.setenv("SVGPU_GLV_PHI64", phi64)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=17 * n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=17 * n)
    B[n // 2] = 0  # identity (0, 0) maps to itself under phi
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp


@pytest.mark.parametrize("path", ["tree", "bucket_tree", "quad", "plain"])
@pytest.mark.parametrize("glv", ["0", "1"])
def test_bucket_reduction_paths(gpu, oracle_cpp, monkeypatch, path, glv):
    """The four bucket reductions -- running sums + in-block subset-sum tree (k_wsum_tree<true> +
    k_group_fin, the default once a window has >= 256 segments), the tree straight over the buckets
    (k_wsum_tree<false>), and k_wsum with the quad-form or whole-addition group sums -- give the
    reference Pippenger's point (msm.rs:238-316), on dense
    random scalars and on sparse ones whose windows leave most buckets / segments / tree blocks empty
    (identity partials at every tree level), device-resident and host-fed."""
    import svgpu
    from svgpu import encoding as enc
    monkeypatch.setenv("SVGPU_GLV", glv)
    monkeypatch.setenv("SVGPU_GROUP_TREE", {"tree": "1", "bucket_tree": "2"}.get(path, "0"))
    monkeypatch.setenv("SVGPU_GROUP_QUAD", "0" if path == "plain" else "1")
    for n, start in ((1 << 16, 5), (70001, 9)):
        B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=start)
        S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=start)
        assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0)), (n, "dense")
    # sparse: small scalars (only the lowest windows' low buckets) and a few huge ones
    n = 1 << 16
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=3)
    rng = np.random.default_rng(11)
    sc = [int(x) for x in rng.integers(0, 1 << 12, n)]
    for i in range(0, n, 4099):
        sc[i] = b.R - 1 - i
    S = enc.scalars_array(sc)
    assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0)), "sparse"
    monkeypatch.setenv("SVGPU_H2D_PIECES", "3")
    assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0)), "sparse host-fed"
    if path == "bucket_tree" and glv == "1":
        # c = 16: 128 tree blocks per window, so k_group_fin sums U_k (k < 8) over two waves
        monkeypatch.delenv("SVGPU_H2D_PIECES")
        n = 1 << 19
        B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=23)
        S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=23)
        assert svgpu.msm_arrays(B, S) == _to_pt(oracle_cpp.msm_pippenger(B, S, 0)), "2^19"


@pytest.mark.parametrize("chain", ["1", "0"])
def test_accumulate_chains(gpu, oracle_cpp, monkeypatch, chain):
    """k_accumulate's two chains (SVGPU_ACC_R29: 9 x 29-bit limbs with the sums stored as the chain's
    own limb records and converted once per bucket by their readers, or 8 x 32-bit limbs), with every
    reader of the stored sums:
    the default tree, the plain k_wsum reduction, host-fed pieces (ADD mode: owner segments start
    from the stored sums), repeated points (the doubling folded into the addition), P + (-P), and
    one skewed bucket (k_fixup's heavy queue), against the reference Pippenger (msm.rs:238-316)."""
    import svgpu
    monkeypatch.setenv("SVGPU_ACC_R29", chain)
    n = 40000
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=77)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=77)
    B[100:3000] = B[99]  # one base repeated with equal scalars: same-bucket doublings
    S[100:3000] = S[99]
    from svgpu import encoding as enc
    x, y = enc.g1_from_limbs(B[5000])
    B[5001] = enc.bases_array([(x, b.P - y)])[0]  # -P with the same scalar: cancels in every bucket
    S[5001] = S[5000]
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp
    monkeypatch.setenv("SVGPU_GROUP_TREE", "0")
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp
    monkeypatch.delenv("SVGPU_GROUP_TREE")
    monkeypatch.setenv("SVGPU_H2D_PIECES", "3")
    n2 = 1 << 18  # host-fed in pieces (from 2^15 points)
    B2 = oracle_cpp.gen_bases(b.SEED_BASES, n2, start=3)
    S2 = oracle_cpp.gen_scalars(b.SEED_SCALARS, n2, start=3)
    S2[: n2 // 2] = S2[0]  # half the points in one bucket per window
    assert svgpu.msm_arrays(B2, S2, svgpu.SV_CANONICAL) == _to_pt(oracle_cpp.msm_pippenger(B2, S2, 0))


@pytest.mark.parametrize("fed", ["device", "host_pieces"])
def test_chain_cancels_and_restarts(gpu, oracle_cpp, monkeypatch, fed):
    """Round 6's chain state is never the identity: a P + (-P) inside a chunk empties it and the next
    point restarts it; a chunk that ends empty stores the identity record (ZZ = 0) that k_fixup, the
    in-block join, the tree and the host-fed pieces' ADD mode must read as such.  All scalars equal
    (every window's entries in ONE bucket), points (A_0, -A_0, A_1, -A_1, ...) plus one extra Z: every
    pair cancels, at every chunk position, and the MSM is s Z; then the pairs reversed (-A_i, A_i)
    and a doubling pair (Z, Z) in the middle.  Against the reference Pippenger (msm.rs:238-316)."""
    import svgpu
    from svgpu import encoding as enc
    n_pairs = (1 << 15) // 2 if fed == "host_pieces" else 2048
    if fed == "host_pieces":
        monkeypatch.setenv("SVGPU_H2D_PIECES", "3")
    A = oracle_cpp.gen_bases(b.SEED_BASES, n_pairs + 1, start=91)
    pts = [enc.g1_from_limbs(r) for r in A]
    z = pts[-1]
    for flip in (False, True):
        seq = []
        for p in pts[:-1]:
            q = b.g1_neg(p)
            seq += [q, p] if flip else [p, q]
        if flip:
            seq[n_pairs: n_pairs] = [z, z]   # a doubling in the middle of the bucket
        seq.append(z)
        B = enc.bases_array(seq)
        S = np.repeat(enc.scalars_array([0x1234567890ABCDEF1234567890ABCDEF]), len(seq), axis=0)
        exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
        assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp, (fed, flip)


@pytest.mark.parametrize("chain", ["1", "0"])
@pytest.mark.parametrize("opt", ["SVGPU_MSM_SPLIT", "SVGPU_FINE_SPLIT", "SVGPU_SORT_FORK"])
def test_optional_pipeline_paths(gpu, oracle_cpp, monkeypatch, opt, chain):
    """The opt-in single-MSM variants kept for A/B -- window halves sorted / accumulated / reduced
    separately (SVGPU_MSM_SPLIT: half B's sort and accumulate on the sort stream, the 29-bit point
    table written by half A's sort only), the two-launch fine sort, the forked fine sort -- with both
    bucket chains, against the reference Pippenger (msm.rs:238-316)."""
    import svgpu
    from svgpu import device as dv
    monkeypatch.setenv(opt, "1")
    monkeypatch.setenv("SVGPU_ACC_R29", chain)
    for n, start in ((1 << 16, 21), (70001, 23)):
        B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=start)
        S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=start)
        exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
        dev = torch.device("cuda", 0)
        Bt = torch.from_numpy(B.view(np.int64)).to(dev)
        St = torch.from_numpy(S.view(np.int64)).to(dev)
        assert dv.msm(Bt, St, svgpu.SV_CANONICAL) == exp, (opt, n, "device")  # the split path's input
        assert svgpu.msm_arrays(B, S) == exp, (opt, n, "host")


@pytest.mark.parametrize("small", ["0", "1"])
@pytest.mark.parametrize("n", [1, 2, 3, 31, 64, 65, 200, 256, 257])
def test_small_msm_path_vs_pipeline(gpu, oracle_cpp, n, small, monkeypatch):
    """MSMs of at most 256 terms take the small path (round 5: window sums on the device, the window
    Horner on the host, msm_batch.hip msm_batch_windows_host); SVGPU_SMALL_MSM=0 keeps the pipeline.
    Both give the reference Pippenger's point -- host-fed in both forms and device-resident -- with a
    zero scalar, an identity base, a repeated point and a cancelling pair mixed in."""
    import svgpu
    from svgpu import device as dv, encoding as enc
    monkeypatch.setenv("SVGPU_SMALL_MSM", small)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=13 * n).copy()
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=13 * n).copy()
    if n >= 4:
        S[0] = 0                      # a zero scalar
        B[1] = 0                      # the identity base (0, 0)
        B[2], S[2] = B[3], S[3]       # a repeated point (same bucket: the doubling case)
    if n >= 6:
        B[5] = enc.bases_array([b.g1_neg(enc.g1_from_limbs(B[4]))])[0]
        S[5] = S[4]                   # P and -P with equal scalars cancel
    exp = _to_pt(oracle_cpp.msm_pippenger(B, S, 0))
    assert svgpu.msm_arrays(B, S, svgpu.SV_CANONICAL) == exp
    Bm = enc.bases_array([enc.g1_from_limbs(r) for r in B], svgpu.SV_MONTGOMERY)
    Sm = enc.scalars_array([enc.limbs_to_int(r) for r in S], svgpu.SV_MONTGOMERY)
    assert svgpu.msm_arrays(Bm, Sm, svgpu.SV_MONTGOMERY) == exp
    Bd = torch.from_numpy(B.view(np.int64)).to(gpu)
    Sd = torch.from_numpy(S.view(np.int64)).to(gpu)
    assert dv.msm(Bd, Sd, svgpu.SV_CANONICAL) == exp
