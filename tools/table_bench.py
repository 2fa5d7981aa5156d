"""Precomputed fixed-base tables: table creation (upload + 2^(8w) P expansion) and the batched
table MSM latency (HBM-resident handle API) for several batch shapes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402

svgpu.init()
dev = torch.device("cuda", 0)
M = svgpu.SV_MONTGOMERY
rows = 4096
Th = dv.gen_bases(dv.empty_bases(rows, dev), 0xBA5E5, 0, svgpu.SV_CANONICAL).cpu().numpy().view(np.uint64)
t0 = time.perf_counter()
tab = svgpu.BaseTable(Th)
print(f"table create ({rows} rows, precompute included): {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
for m in (16, 64, 256, 1024):
    for count in (1, 16, 128, 512):
        n = count * m
        S = dv.gen_scalars(dv.empty_scalars(n, dev), 0x5CA1A75, 0, M)
        idx = torch.randint(0, rows, (n,), dtype=torch.int32, device=dev)
        off = torch.arange(0, n + 1, m, dtype=torch.int64, device=dev)
        tab.msm_batch_device(idx, S, off, M)
        torch.cuda.synchronize()
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            tab.msm_batch_device(idx, S, off, M)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"m={m:5d} count={count:4d}: {ms:8.3f} ms  ({n / ms * 1e3:.3e} terms/s)", flush=True)
