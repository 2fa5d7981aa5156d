"""Config 4 (BASELINE.json): one BN254 G1 MSM of 2^24 points, and its 8-way point split.

* The whole 2^24-point MSM through the C ABI equals the C++ restatement of
  util::msm::multi_scalar_multiplication (msm.rs:238-316; at 2^24 the reference picks c = 19 for one
  chunk, c = 16 per 2^20-point thread chunk) run on the box's host cores.  At this size the GPU
  pipeline takes paths no smaller test reaches: K = 256 entries per accumulate thread, the chunked
  k_fine_sort<true> for every region and the 2^26-entry counting sort.
* The north-star split -- 8 shards of 2^21 points (one per MI355X of a node), each reduced to a
  Jacobian partial by sv_bn254_g1_msm_device and folded in rank order by sv_bn254_g1_fold -- equals
  the whole.  That is exactly what svgpu.parallel.sharded_msm_device does per rank, minus the
  all-gather of the 96-byte partials (covered by tests/test_dist_cpu.py under gloo).

Inputs are generated on the GPU by the seeded generator (sv_gen_*_device, checked against the
oracle's generator in test_gpu_msm.py) and copied to the host for the oracle.
"""
import numpy as np
import pytest
import torch

from oracle import bn254 as b

pytestmark = pytest.mark.gpu

LOG_N = 24
ORACLE_THREADS = 16  # the box's CPU share for one GPU


@pytest.fixture(scope="module")
def inputs_2_24(gpu):
    import svgpu
    from svgpu import device as dv
    n = 1 << LOG_N
    B = dv.gen_bases(dv.empty_bases(n, gpu), b.SEED_BASES, 0, svgpu.SV_CANONICAL)
    S = dv.gen_scalars(dv.empty_scalars(n, gpu), b.SEED_SCALARS, 0, svgpu.SV_CANONICAL)
    torch.cuda.synchronize()
    yield B, S
    del B, S
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def oracle_2_24(inputs_2_24, oracle_cpp):
    B, S = inputs_2_24
    hb = B.cpu().numpy().view(np.uint64)
    hs = S.cpu().numpy().view(np.uint64)
    return b.g1_from_bytes(oracle_cpp.msm_pippenger(hb, hs, ORACLE_THREADS).tobytes())


@pytest.mark.timeout(300)
def test_msm_2_24_vs_oracle(inputs_2_24, oracle_2_24):
    import svgpu
    from svgpu import device as dv
    B, S = inputs_2_24
    got = dv.msm(B, S, svgpu.SV_CANONICAL)
    st = dv.last_msm_stats()
    assert st["entries"] == (1 << LOG_N) * st["num_windows"]
    assert got == oracle_2_24


@pytest.mark.timeout(300)
def test_msm_2_24_eight_shards_fold_to_whole(inputs_2_24, oracle_2_24):
    import svgpu
    from svgpu import device as dv
    B, S = inputs_2_24
    n = B.shape[0]
    G = 8
    parts = []
    for r in range(G):
        lo, hi = r * n // G, (r + 1) * n // G
        parts.append(dv.msm_partial(B[lo:hi], S[lo:hi], svgpu.SV_CANONICAL))
    assert svgpu.fold_partials(parts) == oracle_2_24
    # the fold is order-independent as a group sum, but the rank-order fold is what every rank runs
    assert svgpu.fold_partials(parts[::-1]) == oracle_2_24
