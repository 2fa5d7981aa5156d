import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "snark-verifier-axiom_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libsvgpu's HIP kernels)")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def pt(v):
    return None if v is None else (int(v[0], 16), int(v[1], 16))


def q2(v):
    return None if v is None else ((int(v[0][0], 16), int(v[0][1], 16)), (int(v[1][0], 16), int(v[1][1], 16)))


@pytest.fixture(scope="session")
def golden_msm():
    return load_golden("msm.json")


@pytest.fixture(scope="session")
def golden_decider():
    return load_golden("decider.json")


@pytest.fixture(scope="session")
def oracle_cpp():
    from oracle import cpu_ref
    if not os.path.exists(cpu_ref.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "cpu")])
    cpu_ref.lib()
    return cpu_ref


@pytest.fixture(scope="session")
def gpu():
    """Initialise libsvgpu on the GPU; fails (never skips) when no GPU is usable."""
    import torch
    import svgpu
    assert torch.cuda.is_available(), "GPU test selected but torch sees no GPU"
    assert svgpu.init() >= 1
    return torch.device("cuda:0")
