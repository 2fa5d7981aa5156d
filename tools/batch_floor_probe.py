"""f1 batch (m = 64 terms) latency against the batch size, fused and unfused (SVGPU_BATCH_FUSE):
count = 1 approximates the per-MSM chain floor (one Horner wave), so the gap to count = 128 is
what the batch's bucket waves and their contention with the Horner waves add."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import torch, svgpu
from svgpu import device as dv
svgpu.init()
dev = torch.device("cuda", 0)
M = svgpu.SV_MONTGOMERY
m = 64
Bd = dv.gen_bases(dv.empty_bases(512 * m, dev), 0xBA5E5, 0, M)
Sd = dv.gen_scalars(dv.empty_scalars(512 * m, dev), 0x5CA1A75, 0, M)
torch.cuda.synchronize()
for rnd in range(2):
    for fuse in ("1", "0"):
        os.environ["SVGPU_BATCH_FUSE"] = fuse
        for count in (1, 8, 32, 128, 256):
            off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)
            r0 = dv.msm_batch(Bd, Sd, off, m, M)
            torch.cuda.synchronize()
            ts = []
            for _ in range(15):
                t0 = time.perf_counter(); dv.msm_batch(Bd, Sd, off, m, M); torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(f"fuse={fuse} count={count:4d} m={m}: med {ts[7]*1e3:.3f} ms min {ts[0]*1e3:.3f} ms", flush=True)
