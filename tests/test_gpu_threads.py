"""Re-entrancy contract of the C ABI (SURVEY.md 8b "Threading"; include/svgpu.h): calls may come
concurrently from rayon workers (snark-verifier-sdk/src/util.rs:95-110), so host threads calling
sv_bn254_g1_msm and sv_bn254_kzg_decide at once on one device -- with two DIFFERENT deciding keys,
so the decider's per-key line cache is switched under running kernels -- must each get the
oracle's answer.  ctypes releases the GIL around every foreign call, so the calls overlap.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import bn254 as b

pytestmark = pytest.mark.gpu


def test_concurrent_msm_and_decide_two_keys(gpu, oracle_cpp):
    import svgpu
    from svgpu import encoding as enc
    from svgpu.kzg import decide_arrays
    from svgpu.loader import msm_arrays

    # two deciding keys (different trapdoors); key A's case has a failing accumulator at index 5
    cases = []
    for seed, bad, n in ((0xA11CE, [5], 24), (0xB0B, [], 40)):
        g2, sg2, accs = b.gen_decider_case(n, seed=seed, bad=bad)
        dk = svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2)
        L = enc.bases_array([a[0] for a in accs])
        R = enc.bases_array([a[1] for a in accs])
        cases.append((dk, L, R, bad[0] if bad else -1))
    # deciding A's accumulators against B's lines would fail at index 0: a line-cache race shows
    assert decide_arrays(cases[1][0], cases[0][1], cases[0][2]) == 0

    msms = []
    for k, n in enumerate((777, 5000, 20000)):
        B = oracle_cpp.gen_bases(b.SEED_BASES, n, start=1000 * k)
        S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n, start=3000 * k)
        msms.append((B, S, b.g1_from_bytes(oracle_cpp.msm_pippenger(B, S, 0).tobytes())))

    def job(i):
        if i % 2 == 0:
            dk, L, R, exp = cases[(i // 2) % 2]
            return ("decide", decide_arrays(dk, L, R), exp)
        B, S, exp = msms[(i // 2) % 3]
        return ("msm", msm_arrays(B, S), exp)

    with ThreadPoolExecutor(max_workers=8) as ex:
        results = list(ex.map(job, range(96)))
    bad = [(i, kind) for i, (kind, got, exp) in enumerate(results) if got != exp]
    assert not bad, f"concurrent calls disagreed with the oracle: {bad[:8]}"


def test_concurrent_decide_key_churn(gpu):
    """More distinct keys than the per-device cache holds, decided concurrently: every entry is
    evicted while other calls may still hold it; each call must keep its own lines alive."""
    import svgpu
    from svgpu import encoding as enc
    from svgpu.kzg import decide_arrays

    keys = []
    for j in range(7):
        g2, sg2, accs = b.gen_decider_case(6, seed=0x5EED00 + j, bad=[j % 6])
        keys.append((svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2), enc.bases_array([a[0] for a in accs]),
                     enc.bases_array([a[1] for a in accs]), j % 6))

    def job(i):
        dk, L, R, exp = keys[(i * 3) % len(keys)]
        return decide_arrays(dk, L, R), exp

    with ThreadPoolExecutor(max_workers=6) as ex:
        results = list(ex.map(job, range(84)))
    assert all(got == exp for got, exp in results), results


def test_concurrent_batches_with_big_msms(gpu, oracle_cpp):
    """Batched small MSMs (the fused bucket + Horner launch, whose Horner waves wait on flags of
    their own launch) from several threads at once, beside concurrent 2^20 MSMs on the same GPU:
    at most one fused launch per device is in flight, the rest take the two-kernel path, and every
    call returns the oracle's answer."""
    import svgpu
    from svgpu.loader import msm_arrays
    n = 1 << 20
    BB = oracle_cpp.gen_bases(b.SEED_BASES, n)
    SB = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    big = b.g1_from_bytes(oracle_cpp.msm_pippenger(BB, SB, 0).tobytes())
    batches = []
    for k in range(3):
        sizes = [64] * 128 if k < 2 else [17, 200, 64, 255] * 40
        tot = sum(sizes)
        B = oracle_cpp.gen_bases(b.SEED_BASES, tot, start=50000 * (k + 1))
        S = oracle_cpp.gen_scalars(b.SEED_SCALARS, tot, start=70000 * (k + 1))
        off = [0]
        for m in sizes:
            off.append(off[-1] + m)
        exp = [b.g1_from_bytes(oracle_cpp.msm_pippenger(B[lo:hi], S[lo:hi], 1).tobytes())
               for lo, hi in zip(off[:-1], off[1:])]
        batches.append((B, S, off, exp))

    def job(i):
        if i % 4 == 3:
            return ("msm", msm_arrays(BB, SB) == big)
        B, S, off, exp = batches[i % 3]
        return ("batch", svgpu.msm_batch_arrays(B, S, off) == exp)

    with ThreadPoolExecutor(max_workers=8) as ex:
        results = list(ex.map(job, range(40)))
    bad = [(i, kind) for i, (kind, ok) in enumerate(results) if not ok]
    assert not bad, bad
