"""Child process of tests/test_gpu_msm_config4.py::test_logical_devices_* (not collected by pytest).

Run with SVGPU_DEVICE_MAP set (e.g. "0,0,0,0,0,0,0,0"): libsvgpu then exposes that many logical
devices, and the num_gpus > 1 host entry points -- the path the Rust shim takes with num_gpus = 0 --
run one host thread per logical device (api.cpp for_each_device: own workspace lease, own copy
stream, host fold of the partials / first_fail combine).  Prints one JSON line of results; the
parent compares them with the oracle.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402
from svgpu import encoding as enc  # noqa: E402
from svgpu.kzg import KzgDecidingKey, decide_arrays  # noqa: E402
from oracle import bn254 as b  # noqa: E402


def hexpt(p):
    return None if p is None else [hex(p[0]), hex(p[1])]


def main():
    log_n = int(sys.argv[1])
    ngpu = int(sys.argv[2])
    dev = torch.device("cuda:0")
    out = {"device_count": svgpu.init()}
    n = 1 << log_n
    C = svgpu.SV_CANONICAL
    B = dv.gen_bases(dv.empty_bases(n, dev), b.SEED_BASES, 0, C)
    S = dv.gen_scalars(dv.empty_scalars(n, dev), b.SEED_SCALARS, 0, C)
    torch.cuda.synchronize()
    hB = B.cpu().numpy().view(np.uint64).copy()
    hS = S.cpu().numpy().view(np.uint64).copy()
    del B, S
    torch.cuda.empty_cache()
    out["msm"] = hexpt(svgpu.msm_arrays(hB, hS, C, ngpu))
    out["msm_3"] = hexpt(svgpu.msm_arrays(hB, hS, C, 3))  # uneven split over 3 logical devices
    perm = np.random.default_rng(11).permutation(n).astype(np.uint64)
    refs = svgpu.make_refs(hS.ctypes.data + 32 * perm, hB.ctypes.data + 64 * perm)
    out["msm_refs"] = hexpt(svgpu.msm_refs(refs, C, ngpu))
    del refs, hB, hS
    # decide_all over 256 accumulators sharded 8 ways: failures at 37 and 200 -> first_fail 37
    g2, sg2, accs = b.gen_decider_case(16)
    accs = (accs * 16)[:256]
    bad = [37, 200]
    accs = [((b.g1_add(l, b.G1_GEN), r) if i in bad else (l, r)) for i, (l, r) in enumerate(accs)]
    L = enc.bases_array([a[0] for a in accs])
    R = enc.bases_array([a[1] for a in accs])
    dk = KzgDecidingKey(b.G1_GEN, g2, sg2)
    out["decide_first_fail"] = decide_arrays(dk, L, R, C, ngpu)
    good = b.gen_decider_case(16)[2] * 16
    Lg = enc.bases_array([a[0] for a in good])
    Rg = enc.bases_array([a[1] for a in good])
    out["decide_all_pass"] = decide_arrays(dk, Lg, Rg, C, ngpu)
    print("RESULT " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
