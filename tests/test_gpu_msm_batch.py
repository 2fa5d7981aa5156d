"""Batched small MSMs through the C ABI against the C++ oracle (msm.rs
restatement): ragged sizes, both windows, both forms, the reference's edge suite per MSM,
big-MSM routing, empty-MSM panic, and the config-5 shape (2 x 64 terms) on device buffers."""
import random

import numpy as np
import pytest
import torch

from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def _expected(oracle_cpp, B, S, offsets):
    return [b.g1_from_bytes(oracle_cpp.msm_pippenger(B[lo:hi], S[lo:hi], 1).tobytes())
            for lo, hi in zip(offsets[:-1], offsets[1:])]


def _ragged(oracle_cpp, sizes, seed):
    n = sum(sizes)
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=seed)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=seed)
    offsets = [0]
    for m in sizes:
        offsets.append(offsets[-1] + m)
    return B, S, offsets


@pytest.mark.parametrize("window", ["5", "8"])
def test_ragged_batch_both_windows(gpu, oracle_cpp, monkeypatch, window):
    import svgpu
    monkeypatch.setenv("SVGPU_BATCH_WINDOW_BITS", window)
    sizes = [1, 2, 3, 63, 64, 65, 127, 128, 129, 200, 255, 256, 257, 300, 513, 1023]
    B, S, off = _ragged(oracle_cpp, sizes, 1000)
    assert svgpu.msm_batch_arrays(B, S, off) == _expected(oracle_cpp, B, S, off)


def test_montgomery_form(gpu, oracle_cpp, monkeypatch):
    import svgpu
    monkeypatch.setenv("SVGPU_BATCH_SEQ_MAX", "0")
    from svgpu import encoding as enc
    sizes = [5, 64, 17]
    B, S, off = _ragged(oracle_cpp, sizes, 77)
    exp = _expected(oracle_cpp, B, S, off)
    pts = [enc.g1_from_limbs(r) for r in B]
    sc = [enc.limbs_to_int(r) for r in S]
    Bm, Sm = enc.bases_array(pts, svgpu.SV_MONTGOMERY), enc.scalars_array(sc, svgpu.SV_MONTGOMERY)
    got = svgpu.msm_batch_arrays(Bm, Sm, off, svgpu.SV_MONTGOMERY)
    assert got == exp


def test_edge_suite_per_msm(gpu):
    """zero scalars, identity bases, P and -P, repeated base, r - 1, 2^k, all-equal scalars."""
    import svgpu
    P = b.g1_mul(b.G1_GEN, 987654321)
    Q = b.g1_mul(b.G1_GEN, 5)
    msms = [
        [(0, P), (0, Q)],                                   # -> identity
        [(3, None), (4, P)],                                # identity base
        [(7, P), (7, b.g1_neg(P))],                         # cancels
        [(11, P)] * 40,                                     # repeated base, same scalar
        [(b.R - 1, P), (1, P)],                             # (r-1)P + P = O
        [(1 << k, Q) for k in range(0, 254, 7)],            # powers of two
        [(b.R - 1, Q)] * 70,                                # all-equal, top digits
        [(random.Random(3).randrange(b.R), P) for _ in range(33)],
    ]
    got = svgpu.batch_multi_scalar_multiplication(msms)
    for pairs, g in zip(msms, got):
        assert g == b.native_msm([s for s, _ in pairs], [p for _, p in pairs])


def test_big_msms_route_to_single_pipeline(gpu, oracle_cpp, monkeypatch):
    import svgpu
    monkeypatch.setenv("SVGPU_BATCH_MAX", "100")
    monkeypatch.setenv("SVGPU_BATCH_SEQ_MAX", "0")
    sizes = [10, 3000, 50, 101]
    B, S, off = _ragged(oracle_cpp, sizes, 5000)
    assert svgpu.msm_batch_arrays(B, S, off) == _expected(oracle_cpp, B, S, off)


@pytest.mark.parametrize("sizes", [[64, 64], [30], [12, 40, 7, 256], [300, 64], [64, 1000, 3], [257]])
@pytest.mark.parametrize("host_max", [None, "0"])
def test_tiny_batch_sequential_route(gpu, oracle_cpp, monkeypatch, sizes, host_max):
    """Host-array batches of at most SVGPU_BATCH_SEQ_MAX (4) MSMs: the MSMs of at most 256 terms
    stay in the batch (all-small batches take the small-batch host-Horner route, no id map; mixed
    ones the id-mapped batch kernel), the longer ones run through the single-MSM pipeline.  The
    config-5 shape (two 64-term MSMs) and a proof's few tens-term MSMs (bdfg21.rs:75-78) included."""
    import svgpu
    if host_max is not None:
        monkeypatch.setenv("SVGPU_BATCH_HOST_MAX", host_max)
    B, S, off = _ragged(oracle_cpp, sizes, 9000 + len(sizes))
    assert svgpu.msm_batch_arrays(B, S, off) == _expected(oracle_cpp, B, S, off)


def test_empty_msm_panics(gpu):
    import svgpu
    with pytest.raises(svgpu.ReferencePanic, match="pairs should not be empty"):
        svgpu.batch_multi_scalar_multiplication([[(1, b.G1_GEN)], []])


def test_device_api_config5_shape(gpu, oracle_cpp):
    """64 accumulators -> lhs/rhs MSMs of 64 terms each with [1, r, .., r^63] (accumulation.rs:177-192),
    plus 126 more 64-term MSMs so the batch holds 128 MSMs (a 64-proof aggregation's per-proof pair)."""
    import svgpu
    from svgpu import device as dv
    count, m = 128, 64
    n = count * m
    Bd = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 0, svgpu.SV_MONTGOMERY)
    Sd = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_MONTGOMERY)
    off = torch.arange(0, n + 1, m, dtype=torch.int64, device=gpu)
    out = dv.msm_batch(Bd, Sd, off, m, svgpu.SV_MONTGOMERY)
    torch.cuda.synchronize()
    from svgpu import encoding as enc
    got = [enc.g1_from_limbs(r, svgpu.SV_MONTGOMERY) for r in out.cpu().numpy().view(np.uint64)]
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    assert got == _expected(oracle_cpp, B, S, list(range(0, n + 1, m)))


def test_base_table_host_api(gpu, oracle_cpp):
    """Fixed bases uploaded once, referenced by index from ragged per-proof MSMs (repeated rows,
    identity row, both windows' sizes); then an out-of-table index and a destroyed handle."""
    import svgpu
    T = oracle_cpp.gen_bases(b.SEED_BASES, 300, start=4242)
    T[7] = 0                                           # identity row
    rng = np.random.default_rng(11)
    sizes = [1, 3, 64, 65, 129, 300, 700]
    n = sum(sizes)
    idx = rng.integers(0, 300, n).astype(np.uint32)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=4242)
    off = [0]
    for m in sizes:
        off.append(off[-1] + m)
    with svgpu.BaseTable(T) as tab:
        got = tab.msm_batch_arrays(idx, S, off)
        assert got == _expected(oracle_cpp, T[idx], S, off)
        with pytest.raises(svgpu.ArgumentError):
            tab.msm_batch_arrays(np.array([300], np.uint32), S[:1], [0, 1])
        pairs = [[(5, 1), (7, 2)], [(b.R - 1, 3), (1, 3)]]
        from svgpu import encoding as enc
        assert tab.batch_multi_scalar_multiplication(pairs) == [
            b.native_msm([s for s, _ in p], [enc.g1_from_limbs(T[i]) for _, i in p]) for p in pairs]
        h = tab.handle
    from svgpu import _lib
    out = np.zeros(8, np.uint64)
    assert _lib.lib.sv_bn254_g1_msm_batch_table(h, idx.ctypes.data, S.ctypes.data,
                                                np.array([0, 1], np.uint64).ctypes.data, 1, 0,
                                                out.ctypes.data) == _lib.SV_ERR_ARG


def test_indexed_device_api_matches_direct(gpu, oracle_cpp):
    """Device-buffer table form: a 64-row table referenced by 128 MSMs of 64 terms equals the
    direct batch over the gathered bases; an out-of-range index is caught on the device."""
    import svgpu
    from svgpu import device as dv
    rows, count, m = 64, 128, 64
    n = count * m
    T = dv.gen_bases(dv.empty_bases(rows, gpu), b.SEED_BASES, 0, svgpu.SV_MONTGOMERY)
    Sd = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_MONTGOMERY)
    idx = torch.randint(0, rows, (n,), dtype=torch.int32, device=gpu, generator=None)
    off = torch.arange(0, n + 1, m, dtype=torch.int64, device=gpu)
    got = dv.msm_batch_indexed(T, idx, Sd, off, m)
    ref = dv.msm_batch(T[idx.long()].contiguous(), Sd, off, m)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    from svgpu import encoding as enc
    Th = oracle_cpp.gen_bases(b.SEED_BASES, rows)
    Sh = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    ih = idx.cpu().numpy()
    exp = _expected(oracle_cpp, Th[ih[:4 * m]], Sh[:4 * m], list(range(0, 4 * m + 1, m)))
    assert [enc.g1_from_limbs(r, svgpu.SV_MONTGOMERY) for r in got[:4].cpu().numpy().view(np.uint64)] == exp
    idx[5] = rows
    with pytest.raises(svgpu.ArgumentError):
        dv.msm_batch_indexed(T, idx, Sd, off, m)


@pytest.mark.parametrize("seq_max", ["0", "1000"])
def test_unreduced_base_rejected_on_both_routes(gpu, oracle_cpp, monkeypatch, seq_max):
    """A base coordinate >= p is SV_ERR_ARG whichever route the batch takes (the batched kernel
    and the sequential single-MSM route share the contract of k_to_mont_bases)."""
    import svgpu
    monkeypatch.setenv("SVGPU_BATCH_SEQ_MAX", seq_max)
    B, S, off = _ragged(oracle_cpp, [8, 8, 8, 8, 8, 8], 321)
    B = B.copy()
    B[13, 0:4] = np.array([0xffffffffffffffff] * 4, np.uint64)  # x = 2^256 - 1 >= p
    with pytest.raises(svgpu.ArgumentError):
        svgpu.msm_batch_arrays(B, S, off)


def test_precomputed_table_device_api(gpu, oracle_cpp):
    """Precomputed table rows (2^(8w) P per row, one bucket set per MSM, k_msm_batch_fixed) through
    the HBM-resident handle API: 128 MSMs x 64 terms over a 4096-row table, both forms, against
    the reference Pippenger over the gathered bases; then the edge terms (identity row, zero and
    r - 1 scalars, repeated rows, > 256 terms: several LDS chunks) and an out-of-table index."""
    import svgpu
    from svgpu import encoding as enc
    rows, count, m = 4096, 128, 64
    n = count * m
    Th = oracle_cpp.gen_bases(b.SEED_BASES, rows, start=777)
    Sh = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=777)
    rng = np.random.default_rng(5)
    ih = rng.integers(0, rows, n).astype(np.uint32)
    offs = list(range(0, n + 1, m))
    exp = _expected(oracle_cpp, Th[ih], Sh, offs)
    with svgpu.BaseTable(Th) as tab:
        assert tab.device() == 0
        idx = torch.from_numpy(ih.view(np.int32)).to(gpu)
        off = torch.tensor(offs, dtype=torch.int64, device=gpu)
        Sc = torch.from_numpy(Sh.view(np.int64)).to(gpu)
        got = tab.msm_batch_device(idx, Sc, off, svgpu.SV_CANONICAL)
        torch.cuda.synchronize()
        assert [enc.g1_from_limbs(r) for r in got.cpu().numpy().view(np.uint64)] == exp
        Sm = torch.from_numpy(enc.scalars_array([enc.limbs_to_int(r) for r in Sh[:8 * m]],
                                                svgpu.SV_MONTGOMERY).view(np.int64)).to(gpu)
        gm = tab.msm_batch_device(idx[:8 * m], Sm, off[:9], svgpu.SV_MONTGOMERY)
        assert [enc.g1_from_limbs(r, svgpu.SV_MONTGOMERY) for r in gm.cpu().numpy().view(np.uint64)] == exp[:8]
        bad = idx.clone()
        bad[77] = rows
        with pytest.raises(svgpu.ArgumentError):
            tab.msm_batch_device(bad, Sc, off, svgpu.SV_CANONICAL)
    T2 = Th[:40].copy()
    T2[3] = 0                                            # identity row
    with svgpu.BaseTable(T2) as tab:
        P = [enc.g1_from_limbs(r) for r in T2]
        msms = [
            [(0, 1), (0, 2)],                            # -> identity
            [(5, 3), (9, 4)],                            # identity row
            [(b.R - 1, 6), (1, 6)],                      # (r - 1) P + P = O
            [(11, 7)] * 50,                              # repeated row
            [(1 << k, 8) for k in range(0, 254, 3)],     # powers of two, top windows
            [(int(rng.integers(1, 1 << 62)) * (k + 1) % b.R, k % 40) for k in range(700)],  # 3 LDS chunks
        ]
        got = tab.batch_multi_scalar_multiplication(msms)
        for pairs, g in zip(msms, got):
            assert g == b.native_msm([s for s, _ in pairs], [P[i] for _, i in pairs])


def test_fused_wait_timeout_is_redone(gpu, oracle_cpp, monkeypatch):
    """k_batch_fused's Horner waves wait on window flags of their own launch; a wait that gives up
    (forced here: SVGPU_BATCH_WAIT_SPINS=0) makes the call redo the batch by the two-kernel path and
    still return the oracle's results, never SV_ERR_DEVICE (msm_batch.hip)."""
    import svgpu
    sizes = [64] * 128
    B, S, off = _ragged(oracle_cpp, sizes, 4242)
    exp = _expected(oracle_cpp, B, S, off)
    monkeypatch.setenv("SVGPU_BATCH_WAIT_SPINS", "0")
    assert svgpu.msm_batch_arrays(B, S, off) == exp
    monkeypatch.delenv("SVGPU_BATCH_WAIT_SPINS")
    assert svgpu.msm_batch_arrays(B, S, off) == exp


@pytest.mark.parametrize("host_max", ["0", "64"])
@pytest.mark.parametrize("form", ["canonical", "montgomery"])
def test_device_small_batch_host_horner(gpu, oracle_cpp, monkeypatch, host_max, form):
    """Small plain batches (<= SVGPU_BATCH_HOST_MAX MSMs of <= 256 terms) take the window sums on the
    device and the Horners on the host (one batch inversion for the affine outputs); 0 keeps the
    fused kernel.  Ragged sizes, an all-zero-scalar MSM (identity out), both forms, batches just
    inside and outside the default limit."""
    import svgpu
    from svgpu import device as dv
    from svgpu import encoding as enc
    monkeypatch.setenv("SVGPU_BATCH_HOST_MAX", host_max)
    f = svgpu.SV_MONTGOMERY if form == "montgomery" else svgpu.SV_CANONICAL
    for sizes in ([64], [1, 2, 64, 3], [17] * 64, [5] * 65, [256, 1, 255]):
        B, S, off = _ragged(oracle_cpp, sizes, 123 + len(sizes))
        if len(sizes) > 1:
            S[off[1]:off[2]] = 0  # the second MSM sums to the identity
        exp = _expected(oracle_cpp, B, S, off)
        if f == svgpu.SV_MONTGOMERY:
            B = enc.bases_array([enc.g1_from_limbs(r) for r in B], f)
            S = enc.scalars_array([enc.limbs_to_int(r) for r in S], f)
        Bd = torch.from_numpy(B.view(np.int64)).to(gpu)
        Sd = torch.from_numpy(S.view(np.int64)).to(gpu)
        od = torch.tensor(off, dtype=torch.int64, device=gpu)
        out = dv.msm_batch(Bd, Sd, od, max(sizes), f)
        torch.cuda.synchronize()
        got = [enc.g1_from_limbs(r, f) for r in out.cpu().numpy().view(np.uint64)]
        assert got == exp, sizes
