"""Latency of small MSMs (config-5 shapes) through the device pipeline and the host API."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch, svgpu
from svgpu import device as dv
from oracle import bn254 as ob
svgpu.init()
dev = torch.device("cuda:0")
for n in (8, 32, 64, 256, 1024, 4096):
    B = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, 0)
    S = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, 0)
    dv.msm(B, S)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter(); dv.msm(B, S); ts.append(time.perf_counter() - t0)
    st = dv.last_msm_stats()
    print(f"n={n}: {1e3*np.median(ts):.3f} ms (gpu {st['total_ms']-st['host_ms']:.3f} host {st['host_ms']:.3f}) c={st['window_bits']}", flush=True)
g2, sg2, accs = ob.gen_decider_case(64, seed=0x64)
accs_o = [svgpu.KzgAccumulator(*a) for a in accs]
r = ob.gen_scalar(0x7777, 0)
svgpu.KzgAs.create_proof(accs_o, r)
t0 = time.perf_counter(); acc = svgpu.KzgAs.create_proof(accs_o, r); t1 = time.perf_counter()
dk = svgpu.KzgDecidingKey(ob.G1_GEN, g2, sg2)
svgpu.KzgAs.decide(dk, acc); t2 = time.perf_counter()
print(f"config5 restated: accumulate 64 -> {1e3*(t1-t0):.2f} ms, decide 1 -> {1e3*(t2-t1):.2f} ms", flush=True)
