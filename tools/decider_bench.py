"""Time the KZG decider (256 accumulators) and check verdicts; A/B via SVGPU_DECIDER_1LANE."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch, svgpu
from svgpu import device as dv, encoding as enc
from oracle import bn254 as ob
svgpu.init()
dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
g2, sg2, accs = ob.gen_decider_case(16, seed=ob.SEED_TRAPDOOR, bad=[5])
accs = (accs * ((n + 15) // 16))[:n]
L = torch.from_numpy(enc.bases_array([a[0] for a in accs]).view(np.int64)).to(dev)
R = torch.from_numpy(enc.bases_array([a[1] for a in accs]).view(np.int64)).to(dev)
ff, v, gts = dv.decide(g2, sg2, L, R, want_gt=True)
exp_gt = ob.f12_to_list(ob.decide_gt(g2, sg2, *accs[5]))
print("first_fail", ff, "bad count", n - sum(v), "gt[5] ok", gts[5] == exp_gt, flush=True)
for _ in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    dv.decide(g2, sg2, L, R)
    dt = time.perf_counter() - t0
    print(f"decide n={n}: {dt*1e3:.2f} ms  {2*n/dt:.0f} pairings/s", flush=True)
