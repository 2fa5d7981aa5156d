"""Time the KZG decider (256 accumulators) and check verdicts; A/B builds via SVGPU_LIB."""
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
walls, kers = [], []
for _ in range(20):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    dv.decide(g2, sg2, L, R)
    walls.append(time.perf_counter() - t0)
    kers.append(dv.last_decide_kernel_ms())
walls.sort(); kers.sort()
print(f"decide n={n} [{os.path.basename(svgpu._lib.LIB_PATH)}]: wall min {walls[0]*1e3:.3f} med {walls[10]*1e3:.3f} ms, "
      f"kernel min {kers[0]:.3f} med {kers[10]:.3f} ms", flush=True)
