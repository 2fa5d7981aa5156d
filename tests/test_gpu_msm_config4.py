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


@pytest.mark.timeout(600)
def test_logical_devices_host_paths_8_wide(oracle_2_24):
    """The in-process multi-device path (what the Rust shim gets with num_gpus = 0 on an 8-GPU node:
    api.cpp for_each_device, one host thread + workspace lease + copy stream per device, host fold /
    first_fail combine) run 8-wide on this box's one GPU through SVGPU_DEVICE_MAP=0,...,0:
    sv_bn254_g1_msm(num_gpus=8) and sv_bn254_g1_msm_refs(num_gpus=8) at 2^24 equal the oracle, the
    uneven 3-way split too, and sv_bn254_kzg_decide(num_gpus=8) over 256 accumulators with failures
    at 37 and 200 reports 37 (decider.rs:70-80 try_collect: the first Err)."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT
    env = dict(os.environ, SVGPU_DEVICE_MAP=",".join(["0"] * 8))
    child = os.path.join(ROOT, "tests", "logical_devices_child.py")
    r = subprocess.run([sys.executable, "-u", child, str(LOG_N), "8"], env=env, capture_output=True, text=True,
                       timeout=540)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    exp = [hex(oracle_2_24[0]), hex(oracle_2_24[1])]
    assert res["device_count"] == 8
    assert res["msm"] == exp
    assert res["msm_3"] == exp
    assert res["msm_refs"] == exp
    assert res["decide_first_fail"] == 37
    assert res["decide_all_pass"] == -1
