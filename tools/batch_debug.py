"""Debug: tiny batches through the quad f1 path vs the oracle (1-term MSMs with chosen scalars)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import svgpu  # noqa: E402
from oracle import bn254 as b  # noqa: E402

os.environ["SVGPU_BATCH_SEQ_MAX"] = "0"
svgpu.init()
P = b.g1_mul(b.G1_GEN, 987654321)
Q = b.g1_mul(b.G1_GEN, 5)
cases = [[(1, P)], [(2, P)], [(3, P)], [(17, P)], [(32, P)], [(1 << 40, P)], [(b.R - 1, P)], [(1, P), (1, Q)],
         [(5, P), (7, Q)], [(123456789123456789, P)]]
for q in ("1", "0"):
    os.environ["SVGPU_BATCH_QUAD"] = q
    got = svgpu.batch_multi_scalar_multiplication(cases)
    exp = []
    for msm in cases:
        acc = None
        for s, pt in msm:
            acc = b.g1_add(acc, b.g1_mul(pt, s))
        exp.append(acc)
    print("quad", q, [g == e for g, e in zip(got, exp)], flush=True)
