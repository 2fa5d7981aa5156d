"""Where the bench step's wall time goes outside the GPU phases: the full dv.msm step (ctypes
call + fold + Python point), the bare sv_bn254_g1_msm_device call, and the bench loop's extra
last_msm_stats call, each timed over 60 back-to-back steps at 2^20 (lean events)."""
import ctypes
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import _lib  # noqa: E402
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
gc.disable()
part = _lib.sv_g1_jacobian()
st = torch.cuda.current_stream(dev).cuda_stream
bp, sp = B.data_ptr(), S.data_ptr()
raw = _lib.lib.sv_bn254_g1_msm_device


def bare():
    raw(bp, sp, n, M, 0, st, ctypes.byref(part))


def full():
    dv.msm(B, S, M)


def bench_loop():
    dv.msm(B, S, M)
    dv.last_msm_stats()


for _ in range(30):
    full()
for label, fn in (("bare C call", bare), ("dv.msm", full), ("dv.msm + last_msm_stats", bench_loop),
                  ("bare C call", bare)):
    ts = []
    for _ in range(60):
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e3)
    ts = np.array(ts)
    print(f"{label:28s} mean {ts.mean():.4f} median {np.median(ts):.4f} min {ts.min():.4f} ms", flush=True)
os.environ["SVGPU_MSM_LEAN"] = "0"
full()
print("stats", dv.last_msm_stats(), flush=True)
t = []
for _ in range(2000):
    t0 = time.perf_counter()
    dv.last_msm_stats()
    t.append(time.perf_counter() - t0)
print(f"last_msm_stats alone {np.median(t) * 1e6:.1f} us", flush=True)
