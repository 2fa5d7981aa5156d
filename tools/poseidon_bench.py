"""Throughput of the GPU Poseidon permutation / sponge (t = 3 and 5), HBM-resident states."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402

svgpu.init()
dev = torch.device("cuda", 0)
for t in (3, 5):
    for logn in (14, 18, 20):
        n = 1 << logn
        st = torch.randint(0, 1 << 62, (n * t, 4), dtype=torch.int64, device=dev)
        st[:, 3] &= (1 << 59) - 1
        dv.poseidon_permute(st, t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        reps = 10
        for _ in range(reps):
            dv.poseidon_permute(st, t)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"permute t={t} n=2^{logn}: {ms:.3f} ms  {n / ms * 1e3:.3e} perms/s", flush=True)
