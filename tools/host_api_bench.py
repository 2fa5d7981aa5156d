"""Host-buffer MSM timing at 2^20: sv_bn254_g1_msm (pageable Montgomery arrays, the zero-copy
halo2curves layout) per SVGPU_H2D_PIECES, and sv_bn254_g1_msm_refs (shuffled references: the
NativeLoader pair shape, gather included), against the device-resident MSM of the same input."""
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


def t(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, r


svgpu.init()
dev = torch.device("cuda:0")
log_n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 1 << log_n
M = svgpu.SV_MONTGOMERY
Bd = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0, M)
Sd = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0, M)
torch.cuda.synchronize()
B = Bd.cpu().numpy().view(np.uint64).copy()
S = Sd.cpu().numpy().view(np.uint64).copy()
dms, ref = t(lambda: (dv.msm(Bd, Sd, M), torch.cuda.synchronize())[0])
print(f"device-resident  {dms:7.3f} ms")
specs = sys.argv[2:] or ["", "SVGPU_H2D_PIECES=1", "SVGPU_H2D_PIECES=2", "SVGPU_H2D_PIECES=4",
                         "SVGPU_H2D_PIECES=6", "SVGPU_H2D_PIECES=8", "SVGPU_H2D_SPLIT=1,1,2,3,3,3,3",
                         "SVGPU_H2D_SPLIT=1,2,3,3,3,2", "SVGPU_H2D_SPLIT=2,3,3,3,3,2",
                         "SVGPU_H2D_SPLIT=1,2,2,3,3,3,2"]
rng = np.random.default_rng(1)
perm = rng.permutation(n)
rf_shuf = svgpu.make_refs(S.ctypes.data + 32 * perm.astype(np.uint64), B.ctypes.data + 64 * perm.astype(np.uint64))
for spec in specs:
    for k in ("SVGPU_H2D_PIECES", "SVGPU_H2D_SPLIT", "SVGPU_GLV", "SVGPU_H2D_STAGE", "SVGPU_H2D_RING", "SVGPU_H2D_RING_SLOTS"):
        os.environ.pop(k, None)
    for kv in filter(None, spec.split(" ")):
        k, v = kv.split("=")
        os.environ[k] = v
    ms, r = t(lambda: svgpu.msm_arrays(B, S, M))
    rms, rr = t(lambda: svgpu.msm_refs(rf_shuf, M))
    print(f"host [{spec or 'default'}]  {ms:7.3f} ms  x{ms / dms:.2f}  ok={r == ref}   refs {rms:7.3f} ms  "
          f"x{rms / dms:.2f}  ok={rr == ref}", flush=True)
for k in ("SVGPU_H2D_PIECES", "SVGPU_H2D_SPLIT", "SVGPU_GLV", "SVGPU_H2D_STAGE", "SVGPU_H2D_RING", "SVGPU_H2D_RING_SLOTS"):
    os.environ.pop(k, None)
rng = np.random.default_rng(1)
perm = rng.permutation(n)
sp = S.ctypes.data + 32 * perm.astype(np.uint64)
bp = B.ctypes.data + 64 * perm.astype(np.uint64)
rf = svgpu.make_refs(sp, bp)
ms, r = t(lambda: svgpu.msm_refs(rf, M))
print(f"refs (shuffled)  {ms:7.3f} ms  x{ms / dms:.2f}  ok={r == ref}")
sp = S.ctypes.data + 32 * np.arange(n, dtype=np.uint64)
bp = B.ctypes.data + 64 * np.arange(n, dtype=np.uint64)
rf = svgpu.make_refs(sp, bp)
ms, r = t(lambda: svgpu.msm_refs(rf, M))
print(f"refs (in order)  {ms:7.3f} ms  x{ms / dms:.2f}  ok={r == ref}")
