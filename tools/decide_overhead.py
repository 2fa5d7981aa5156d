"""Per-call overhead of the device decider (256 accumulators): the Python wrapper before/after the
round-5 trim (ctypes verdict array + list(), content-keyed G2 cache vs numpy verdicts + identity
cache) and the kernel timing events on/off (SVGPU_DECIDE_EVENTS), interleaved rounds, one process."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch, svgpu
from svgpu import device as dv, encoding as enc, _lib
from oracle import bn254 as ob
svgpu.init()
dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
g2, sg2, accs = ob.gen_decider_case(16, seed=ob.SEED_TRAPDOOR)
accs = (accs * ((n + 15) // 16))[:n]
L = torch.from_numpy(enc.bases_array([a[0] for a in accs]).view(np.int64)).to(dev)
R = torch.from_numpy(enc.bases_array([a[1] for a in accs]).view(np.int64)).to(dev)


def old_decide(g2, s_g2, lhs, rhs, form=_lib.SV_CANONICAL):
    n = lhs.shape[0]
    d = dv._dev_index(lhs)
    ff = ctypes.c_int32(-2)
    verdicts = (ctypes.c_int32 * n)()
    key1, key2 = (dv._frozen(g2), form), (dv._frozen(s_g2), form)
    g2s, sg2s = dv._G2_CACHE[key1], dv._G2_CACHE[key2]
    _lib.check(_lib.lib.sv_bn254_kzg_decide_device(
        ctypes.byref(g2s), ctypes.byref(sg2s), lhs.data_ptr(), rhs.data_ptr(), n, form, d,
        dv._stream_handle(lhs.device), ctypes.byref(ff), ctypes.cast(verdicts, ctypes.c_void_p), None),
        "sv_bn254_kzg_decide_device")
    return ff.value, list(verdicts), None


ref = dv.decide(g2, sg2, L, R)
assert old_decide(g2, sg2, L, R) == ref and ref[0] == -1
res = {}
for rnd in range(3):
    for name, fn in (("old", old_decide), ("new", dv.decide)):
        for ev in ("1", "0"):
            os.environ["SVGPU_DECIDE_EVENTS"] = ev
            fn(g2, sg2, L, R)
            torch.cuda.synchronize()
            ts = []
            for _ in range(100):
                t0 = time.perf_counter()
                r = fn(g2, sg2, L, R)
                ts.append(time.perf_counter() - t0)
            assert r == ref
            ts.sort()
            res.setdefault((name, ev), []).append(ts[50] * 1e3)
for k, v in res.items():
    print(f"decide n={n} wrapper={k[0]} events={k[1]}: median per call " + " / ".join(f"{x:.4f}" for x in v) + " ms",
          flush=True)
