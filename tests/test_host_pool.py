"""Host worker pool (csrc/hostpool.cpp) under ThreadSanitizer: back-to-back host_parallel_for jobs
from several caller threads, alternating 2-slice and pool-wide jobs (the sv_bn254_kzg_accumulate /
sv_bn254_g1_msm_refs mix).  CPU only; the binary is built by tests/native/Makefile (build())."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BIN = os.path.join(NATIVE, "build", "pool_stress_tsan")


@pytest.fixture(scope="module")
def stress_bin():
    r = subprocess.run(["make", "-s", "-C", NATIVE, "build/pool_stress_tsan"], capture_output=True, text=True)
    if r.returncode != 0 or not os.path.exists(BIN):
        pytest.skip("ThreadSanitizer build unavailable: " + r.stderr[-400:])
    return BIN


@pytest.mark.parametrize("callers,threads", [(2, 16), (4, 16), (3, 5)])
def test_pool_no_race_no_lost_slices(stress_bin, callers, threads):
    env = dict(os.environ, SVGPU_HOST_THREADS=str(threads), TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([stress_bin, str(callers), "1500"], capture_output=True, text=True, env=env, timeout=280)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-3000:]
    assert "bad=0 late=0" in r.stdout
