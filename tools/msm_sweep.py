"""Sweep MSM tuning knobs (SVGPU_WINDOW_BITS, SVGPU_ACC_K) on one GPU; checks every result."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import torch, svgpu
from svgpu import device as dv
from oracle import bn254 as ob
svgpu.init()
dev = torch.device("cuda:0")
log_ns = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "20").split(",")]
for log_n in log_ns:
    n = 1 << log_n
    B = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0)
    S = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0)
    torch.cuda.synchronize()
    ref = None
    for c in [int(x) for x in os.environ.get("SWEEP_C", "14,15,16").split(",")]:
        for K in [int(x) for x in os.environ.get("SWEEP_K", "32,64,128").split(",")]:
            os.environ["SVGPU_WINDOW_BITS"] = str(c)
            if K: os.environ["SVGPU_ACC_K"] = str(K)
            else: os.environ.pop("SVGPU_ACC_K", None)
            r = dv.msm(B, S)
            if ref is None: ref = r
            ts = []
            for _ in range(5):
                t0 = time.perf_counter(); r2 = dv.msm(B, S); ts.append(time.perf_counter() - t0)
            st = dv.last_msm_stats()
            print(f"2^{log_n} c={c} K={K}: {1e3*min(ts):.3f} ms ok={r == ref == r2} acc={st['accumulate_ms']:.3f} "
                  f"sort={st['sort_ms']:.3f} fix={st['fixup_ms']:.3f} red={st['reduce_ms']:.3f} host={st['host_ms']:.3f}",
                  flush=True)
