"""Host-buffer MSMs (sv_bn254_g1_msm on pageable Montgomery arrays, then sv_bn254_g1_msm_refs on
shuffled references; 2^20, four calls each) for a
rocprofv3 --kernel-trace --memory-copy-trace timeline of the piece pipeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import svgpu  # noqa: E402
from svgpu import device as dv  # noqa: E402
from oracle import bn254 as ob  # noqa: E402

svgpu.init()
dev = torch.device("cuda:0")
n = 1 << 20
M = svgpu.SV_MONTGOMERY
Bd = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0, M)
Sd = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0, M)
torch.cuda.synchronize()
B = Bd.cpu().numpy().view(np.uint64).copy()
S = Sd.cpu().numpy().view(np.uint64).copy()
for _ in range(4):
    svgpu.msm_arrays(B, S, M)
# then the reference-shaped entry point (shuffled references: the gather is inside the call)
perm = np.random.default_rng(1).permutation(n).astype(np.uint64)
refs = svgpu.make_refs(S.ctypes.data + 32 * perm, B.ctypes.data + 64 * perm)
for _ in range(4):
    svgpu.msm_refs(refs, M)
