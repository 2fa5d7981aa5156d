"""Per-step wall times of the bench step (dv.msm at 2^20, lean events), to compare the mean the
bench reports with the median the sweeps report."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import gc  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402
from oracle import bn254 as ob  # noqa: E402

svgpu.init()
dev = torch.device("cuda:0")
n = 1 << 20
M = svgpu.SV_MONTGOMERY
B = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0, M)
S = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0, M)
torch.cuda.synchronize()
os.environ["SVGPU_MSM_LEAN"] = "1"
for label, gc_off in (("gc on", False), ("gc off", True)):
    if gc_off:
        gc.disable()
    for _ in range(5):
        dv.msm(B, S, M)
    ts, acc = [], []
    for _ in range(40):
        t0 = time.perf_counter()
        dv.msm(B, S, M)
        ts.append((time.perf_counter() - t0) * 1e3)
        acc.append(dv.last_msm_stats()["accumulate_ms"])
    ts = np.array(ts)
    print(f"{label}: mean {ts.mean():.3f} median {np.median(ts):.3f} min {ts.min():.3f} max {ts.max():.3f} ms; "
          f"acc mean {np.mean(acc):.3f} median {np.median(acc):.3f}")
    print("  steps:", " ".join(f"{x:.2f}" for x in ts))
    gc.enable()
