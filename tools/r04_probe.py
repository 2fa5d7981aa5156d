"""Round-4 probe: config-5 latency split (host transcript + accumulate + decide) and the batched
small-MSM kernel with / without the fused launch."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import _lib, device as dv, encoding as enc  # noqa: E402
from oracle import bn254 as ob  # noqa: E402

svgpu.init()


def med(fn, reps=10):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


g2, sg2, accs = ob.gen_decider_case(64, seed=ob.SEED_TRAPDOOR)
inst = [svgpu.KzgAccumulator(a[0], a[1]) for a in accs]
dk = svgpu.KzgDecidingKey(ob.G1_GEN, g2, sg2)
L = enc.bases_array([a[0] for a in accs])
R = enc.bases_array([a[1] for a in accs])
ol, orr = _lib.sv_g1_affine(), _lib.sv_g1_affine()
rr = np.zeros(4, np.uint64)
r = ob.gen_scalar(ob.SEED_SCALARS, 1 << 30)
rs = enc.fe_struct(r)
print("abi create_proof  %.3f ms" % med(lambda: _lib.lib.sv_bn254_kzg_create_proof(
    L.ctypes.data, R.ctypes.data, 64, 0, 0, ctypes.byref(ol), ctypes.byref(orr), None, rr.ctypes.data)))
print("abi accumulate    %.3f ms" % med(lambda: _lib.lib.sv_bn254_kzg_accumulate(
    L.ctypes.data, R.ctypes.data, 64, ctypes.byref(rs), 0, 0, ctypes.byref(ol), ctypes.byref(orr))))
print("mirror create_proof(transcript) %.3f ms" % med(lambda: svgpu.KzgAs.create_proof(inst, svgpu.PoseidonTranscript())))
print("mirror create_proof(r)          %.3f ms" % med(lambda: svgpu.KzgAs.create_proof(inst, r)))
acc = svgpu.KzgAs.create_proof(inst)
print("mirror decide                   %.3f ms" % med(lambda: svgpu.KzgAs.decide(dk, acc)))
print("python bases_array x2           %.3f ms" % med(lambda: (enc.bases_array([a.lhs for a in inst]),
                                                              enc.bases_array([a.rhs for a in inst]))))

dev = torch.device("cuda", 0)
M = svgpu.SV_MONTGOMERY
count, m = 128, 64
B = dv.gen_bases(dv.empty_bases(count * m, dev), ob.SEED_BASES, 0, M)
S = dv.gen_scalars(dv.empty_scalars(count * m, dev), ob.SEED_SCALARS, 0, M)
off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)


def batch():
    dv.msm_batch(B, S, off, m, M)
    torch.cuda.synchronize()


for fuse in ("1", "0"):
    os.environ["SVGPU_BATCH_FUSE"] = fuse
    print("msm_batch 128 x 64 fuse=%s  %.3f ms" % (fuse, med(batch)))
