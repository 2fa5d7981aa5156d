"""Time the 2^k MSM under several tuning-env settings (one process; every result checked equal).
Usage: python tools/msm_sweep_env.py LOG_N 'SVGPU_GLV=1,SVGPU_ACC_K=64' 'SVGPU_GLV=0' ..."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import torch, svgpu
from svgpu import device as dv
from oracle import bn254 as ob
svgpu.init()
dev = torch.device("cuda:0")
arg = sys.argv[1]  # LOG_N, or n=COUNT for an arbitrary size
n = int(arg[2:]) if arg.startswith("n=") else 1 << int(arg)
log_n = arg
B = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0)
S = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0)
torch.cuda.synchronize()
KEYS = ("SVGPU_HIST_PF", "SVGPU_GLV", "SVGPU_MSM_LEAN", "SVGPU_ACC_K", "SVGPU_RED_LOG", "SVGPU_WINDOW_BITS", "SVGPU_GLV_MAX_LOG", "SVGPU_SORT_E32", "SVGPU_GROUP_P", "SVGPU_GLV_PHI64", "SVGPU_SORT_FORK", "SVGPU_SORT_HALVES")
BASE = {k: os.environ[k] for k in KEYS if k in os.environ}
ref = None
for rnd in range(int(os.environ.get("SWEEP_ROUNDS", "2"))):
    for spec in sys.argv[2:]:
        for k in KEYS:  # back to the settings the script was started with
            if k in BASE:
                os.environ[k] = BASE[k]
            else:
                os.environ.pop(k, None)
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            os.environ[k] = v
        r = dv.msm(B, S)
        ref = r if ref is None else ref
        ts = []
        sts = []
        for _ in range(int(os.environ.get("SWEEP_REPS", "7"))):
            t0 = time.perf_counter(); r2 = dv.msm(B, S); ts.append(time.perf_counter() - t0)
            sts.append(dv.last_msm_stats())
        # stage times: the median over the timed calls (the last call's alone is noisy)
        st = {k: (sorted(x[k] for x in sts)[len(sts) // 2] if isinstance(sts[0][k], float) else sts[-1][k])
              for k in sts[-1]}
        ts.sort()
        print(f"2^{log_n} [{spec}] c={st['window_bits']} W={st['num_windows']}: med {1e3*ts[len(ts)//2]:.3f} min {1e3*ts[0]:.3f} ms "
              f"ok={r == ref == r2} digits={st['digits_ms']:.3f} sort={st['sort_ms']:.3f} acc={st['accumulate_ms']:.3f} "
              f"fix={st['fixup_ms']:.3f} red={st['reduce_ms']:.3f} host={st['host_ms']:.3f}", flush=True)
