"""One f1 batch shape (bench.py's msm_batch row): 128 MSMs x 64 terms, plain bases, median of 9."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402
from oracle import bn254 as ob  # noqa: E402

svgpu.init()
dev = torch.device("cuda", 0)
M = svgpu.SV_MONTGOMERY
count, m = int(os.environ.get("BATCH_COUNT", 128)), int(os.environ.get("BATCH_TERMS", 64))
B = dv.gen_bases(dv.empty_bases(count * m, dev), ob.SEED_BASES, 0, M)
S = dv.gen_scalars(dv.empty_scalars(count * m, dev), ob.SEED_SCALARS, 0, M)
off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)
ref = dv.msm_batch(B, S, off, m, M)
ts = []
for _ in range(9):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = dv.msm_batch(B, S, off, m, M)
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
print(f"{count} x {m}: median {np.median(ts) * 1e3:.3f} ms, same={bool(torch.equal(r, ref))}")
