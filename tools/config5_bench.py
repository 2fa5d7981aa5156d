"""Config 5 latency split: KzgAs::create_proof (two 64-term MSMs with r^i) and one decide.

python tools/config5_bench.py [reps]   (also used under rocprofv3 --kernel-trace --memory-copy-trace;
tools/config5_trace.py then prints one iteration's timeline)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "snark-verifier-axiom_amd")]
import numpy as np  # noqa: E402

import svgpu  # noqa: E402
from oracle import bn254 as ob  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
svgpu.init()
g2, sg2, accs = ob.gen_decider_case(64, seed=ob.SEED_TRAPDOOR)
r = ob.gen_scalar(ob.SEED_SCALARS, 1 << 30)
inst = [svgpu.KzgAccumulator(a[0], a[1]) for a in accs]
dk = svgpu.KzgDecidingKey(ob.G1_GEN, g2, sg2)


def med(fn):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, out


ms_acc, acc = med(lambda: svgpu.KzgAs.create_proof(inst, r))
ms_dec, _ = med(lambda: svgpu.KzgAs.decide(dk, acc))
ms_tr, acc_t = med(lambda: svgpu.KzgAs.create_proof(inst, svgpu.PoseidonTranscript()))
ms_all, _ = med(lambda: svgpu.KzgAs.decide(dk, svgpu.KzgAs.create_proof(inst, svgpu.PoseidonTranscript())))
(el, er), r_exp, _ = ob.create_proof(accs)
print(f"accumulate(r given) {ms_acc:.3f} ms  create_proof(transcript) {ms_tr:.3f} ms  decide(1) {ms_dec:.3f} ms  "
      f"config5 end-to-end {ms_all:.3f} ms  parity {(acc.lhs, acc.rhs) == ob.accumulate(accs, r)} "
      f"{(acc_t.lhs, acc_t.rhs) == (el, er)}")
