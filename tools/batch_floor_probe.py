"""f1 batch (m = 64 terms) latency against the batch size, fused and unfused (SVGPU_BATCH_FUSE):
count = 1 approximates the per-MSM chain floor (one Horner wave), so the gap to count = 128 is
what the batch's bucket waves and their contention with the Horner waves add.
`python tools/batch_floor_probe.py host`: the small-batch host-Horner route (SVGPU_BATCH_HOST_MAX
0 = never vs 1000 = always) against the batch size instead, to place the crossover."""
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
host = len(sys.argv) > 1 and sys.argv[1] == "host"
key = "SVGPU_BATCH_HOST_MAX" if host else "SVGPU_BATCH_FUSE"
for rnd in range(2):
    for val in (("0", "1000") if host else ("1", "0")):
        os.environ[key] = val
        if not host:
            os.environ["SVGPU_BATCH_HOST_MAX"] = "0"  # the device kernels at every size
        for count in ((1, 2, 8, 16, 32, 48, 64, 96, 128) if host else (1, 8, 32, 128, 256)):
            off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)
            r0 = dv.msm_batch(Bd, Sd, off, m, M)
            torch.cuda.synchronize()
            ts = []
            for _ in range(15):
                t0 = time.perf_counter(); dv.msm_batch(Bd, Sd, off, m, M); torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(f"{key}={val} count={count:4d} m={m}: med {ts[7]*1e3:.3f} ms min {ts[0]*1e3:.3f} ms", flush=True)
