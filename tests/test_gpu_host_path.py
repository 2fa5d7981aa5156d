"""Host-buffer MSM entry points (the ones the Rust shim binds) against the C++
oracle: sv_bn254_g1_msm streams its pageable inputs HBM-ward in pieces (SVGPU_H2D_PIECES /
SVGPU_H2D_SPLIT), each piece sorted on a second stream and accumulated into the one bucket set
(pieces after the first add into it) while later pieces are in flight; and
sv_bn254_g1_msm_refs takes NativeLoader's own shape -- an array of (&Fr, &G1Affine) references
(native.rs:61-71) -- and gathers the referenced values itself."""
import numpy as np
import pytest

from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def _case(oracle_cpp, n, start):
    B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=start)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=start)
    return B, S, b.g1_from_bytes(oracle_cpp.msm_pippenger(B, S, 0).tobytes())


@pytest.mark.parametrize("pieces", ["1", "2", "3", "4", "8", "16"])
def test_host_msm_pieces(gpu, oracle_cpp, monkeypatch, pieces):
    import svgpu
    monkeypatch.setenv("SVGPU_H2D_PIECES", pieces)
    for n, start in ((1, 7), (100, 11), (5000, 13), (65539, 17), (300001, 19)):
        B, S, exp = _case(oracle_cpp, n, start)
        assert svgpu.msm_arrays(B, S) == exp, (n, pieces)


@pytest.mark.parametrize("split", [None, "2,2,3,3,3,3", "1,7,1", "5,1", "1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1"])
def test_host_msm_split_schedules(gpu, oracle_cpp, monkeypatch, split):
    """Uneven piece schedules (the default is 2,2,3,3,3,3 from 2^18 points): every piece's own chunk
    length K, its own sorted entries, and the add-into accumulate / fixup for pieces after the first,
    in both input forms (Montgomery bases are only checked, canonical ones converted per piece)."""
    import svgpu
    monkeypatch.delenv("SVGPU_H2D_PIECES", raising=False)
    if split is None:
        monkeypatch.delenv("SVGPU_H2D_SPLIT", raising=False)
    else:
        monkeypatch.setenv("SVGPU_H2D_SPLIT", split)
    for n, start in ((4096 * 3 + 5, 37), (40000, 41), (262147, 43)):
        B, S, exp = _case(oracle_cpp, n, start)
        assert svgpu.msm_arrays(B, S) == exp, (n, split)
    Bm, Sm = _to_mont(B), _to_mont(S, scalar=True)
    assert svgpu.msm_arrays(Bm, Sm, svgpu.SV_MONTGOMERY) == exp, split


def _to_mont(a, scalar=False):
    """Canonical limbs -> Montgomery limbs (x R mod p for coordinates, mod r for scalars); identity
    points stay (0, 0)."""
    mod = b.R if scalar else b.P
    words = a.reshape(-1, 4)
    out = np.zeros_like(words)
    for i, w in enumerate(words):
        v = int(w[0]) | int(w[1]) << 64 | int(w[2]) << 128 | int(w[3]) << 192
        m = v * (1 << 256) % mod
        out[i] = [(m >> (64 * k)) & (2**64 - 1) for k in range(4)]
    return out.reshape(a.shape)


@pytest.mark.parametrize("n", [5000, 20000, 300001])
def test_unreduced_montgomery_bases_rejected(gpu, oracle_cpp, monkeypatch, n):
    """A Montgomery-form base coordinate >= p is SV_ERR_ARG on every path (the 2p-domain adds assume
    reduced inputs): device-resident with and without the GLV table, host-fed with one piece and with
    several (GLV: checked by the piece's table pass; without GLV by k_check_bases)."""
    import torch
    import svgpu
    from svgpu import device as dv
    B, S, _ = _case(oracle_cpp, n, 47)
    Sm = _to_mont(S, scalar=True)
    for coord in (0, 4):  # x, y
        Bbad = B.copy()
        Bbad[n // 2, coord:coord + 4] = np.array([0xffffffffffffffff] * 3 + [0x3fffffffffffffff], np.uint64)
        dB = torch.from_numpy(Bbad.view(np.int64)).to(gpu)
        dS = torch.from_numpy(Sm.view(np.int64)).to(gpu)
        with pytest.raises(svgpu.ArgumentError):
            dv.msm(dB, dS, svgpu.SV_MONTGOMERY)
        for glv in ("1", "0"):
            monkeypatch.setenv("SVGPU_GLV", glv)
            for pieces in ("1", "3"):
                monkeypatch.setenv("SVGPU_H2D_PIECES", pieces)
                with pytest.raises(svgpu.ArgumentError):
                    svgpu.msm_arrays(Bbad, Sm, svgpu.SV_MONTGOMERY)
        monkeypatch.delenv("SVGPU_GLV")
        monkeypatch.delenv("SVGPU_H2D_PIECES")


def test_host_msm_2_20_montgomery(gpu, oracle_cpp):
    """Config 2 through the host API in halo2curves' Montgomery layout (zero-copy from Rust)."""
    import torch
    import svgpu
    from svgpu import device as dv
    n = 1 << 20
    Bm = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 0, svgpu.SV_MONTGOMERY).cpu().numpy().view(np.uint64)
    Sm = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_MONTGOMERY).cpu().numpy().view(np.uint64)
    Bc = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 0, svgpu.SV_CANONICAL).cpu().numpy().view(np.uint64)
    Sc = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_CANONICAL).cpu().numpy().view(np.uint64)
    torch.cuda.synchronize()
    exp = b.g1_from_bytes(oracle_cpp.msm_pippenger(Bc, Sc, 16).tobytes())
    assert svgpu.msm_arrays(Bm, Sm, svgpu.SV_MONTGOMERY) == exp
    assert svgpu.msm_arrays(Bc, Sc, svgpu.SV_CANONICAL) == exp


def test_host_msm_edges_and_errors(gpu, oracle_cpp):
    import svgpu
    B, S, _ = _case(oracle_cpp, 20000, 23)
    S0 = np.zeros_like(S)
    assert svgpu.msm_arrays(B, S0) is None                       # all-zero scalars -> identity
    Bi = B.copy()
    Bi[::3] = 0                                                   # identity bases mixed in
    assert svgpu.msm_arrays(Bi, S) == b.g1_from_bytes(oracle_cpp.msm_pippenger(Bi, S, 0).tobytes())
    Sbad = S.copy()
    Sbad[12345] = np.array([0xffffffffffffffff] * 4, np.uint64)   # >= r
    with pytest.raises(svgpu.ArgumentError):
        svgpu.msm_arrays(B, Sbad)
    Bbad = B.copy()
    Bbad[19999, 4:8] = np.array([0xffffffffffffffff] * 4, np.uint64)  # y >= p (canonical path)
    with pytest.raises(svgpu.ArgumentError):
        svgpu.msm_arrays(Bbad, S)


@pytest.mark.parametrize("n", [1, 777, 70001])
def test_refs_gather_matches_oracle(gpu, oracle_cpp, n):
    """References in a shuffled order, some pairs aliasing the same base / scalar."""
    import svgpu
    B, S, _ = _case(oracle_cpp, n, 29)
    rng = np.random.default_rng(n)
    perm = rng.permutation(n)
    alias = rng.integers(0, n, size=n)
    pick_b = np.where(rng.random(n) < 0.1, alias, perm)         # 10 % of pairs reuse another base
    pick_s = perm[::-1].copy()
    sp = S.ctypes.data + 32 * pick_s.astype(np.uint64)
    bp = B.ctypes.data + 64 * pick_b.astype(np.uint64)
    exp = b.g1_from_bytes(oracle_cpp.msm_pippenger(B[pick_b], S[pick_s], 0).tobytes())
    assert svgpu.msm_refs(svgpu.make_refs(sp, bp)) == exp


def test_refs_null_and_empty(gpu, oracle_cpp):
    import svgpu
    B, S, _ = _case(oracle_cpp, 10, 31)
    sp = S.ctypes.data + 32 * np.arange(10, dtype=np.uint64)
    bp = B.ctypes.data + 64 * np.arange(10, dtype=np.uint64)
    bp[4] = 0
    with pytest.raises(svgpu.ArgumentError):
        svgpu.msm_refs(svgpu.make_refs(sp, bp))
    with pytest.raises(svgpu.ReferencePanic, match="pairs should not be empty"):
        svgpu.msm_refs(svgpu.make_refs(sp[:0], bp[:0]))
