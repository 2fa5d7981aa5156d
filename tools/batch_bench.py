"""Latency / throughput of batched small MSMs (device API) vs one-at-a-time single MSMs."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402

svgpu.init()
dev = torch.device("cuda", 0)
M = svgpu.SV_MONTGOMERY
NMAX = 512 * 1024
Bd = dv.gen_bases(dv.empty_bases(NMAX, dev), 0xBA5E5, 0, M)
Sd = dv.gen_scalars(dv.empty_scalars(NMAX, dev), 0x5CA1A75, 0, M)
torch.cuda.synchronize()


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


for m in (16, 64, 256, 1024):
    for count in (1, 2, 16, 128, 512):
        if count * m > NMAX:
            continue
        off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)
        ms = timeit(lambda: dv.msm_batch(Bd, Sd, off, m, M))
        line = f"m={m:5d} count={count:4d}: batch {ms:8.3f} ms  ({count * m / ms * 1e3:.3e} terms/s)"
        if count <= 16:
            seq = timeit(lambda: [dv.msm(Bd[i * m:(i + 1) * m], Sd[i * m:(i + 1) * m], M) for i in range(count)], 2)
            line += f"   sequential single-MSM {seq:8.3f} ms"
        print(line, flush=True)
