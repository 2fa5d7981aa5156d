"""First on-GPU check: generator parity, MSM parity vs the Python oracle, decider parity, 2^20 timing."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
sys.path.insert(0, ROOT)
import torch
import svgpu
from svgpu import device as dv, encoding as enc
from oracle import bn254 as b

print("devices", svgpu.init(), svgpu.version(), flush=True)
dev = torch.device("cuda:0")
ok = True
for form in (svgpu.SV_CANONICAL, svgpu.SV_MONTGOMERY):
    for n in (1, 2, 3, 17, 64, 300):
        B = dv.gen_bases(dv.empty_bases(n, dev), b.SEED_BASES, 0, form)
        S = dv.gen_scalars(dv.empty_scalars(n, dev), b.SEED_SCALARS, 0, form)
        torch.cuda.synchronize()
        hb = B.cpu().numpy().view("uint64"); hs = S.cpu().numpy().view("uint64")
        pts = [enc.g1_from_limbs(hb[i], form) for i in range(n)]
        scs = [enc._from_form(enc.limbs_to_int(hs[i]), b.R, form) for i in range(n)]
        gen_ok = pts == b.gen_bases(b.SEED_BASES, n) and scs == b.gen_scalars(b.SEED_SCALARS, n)
        got = dv.msm(B, S, form)
        exp = b.pippenger_msm(scs, pts)
        host_api = svgpu.msm_arrays(hb, hs, form)
        r = gen_ok and got == exp and host_api == exp
        ok &= r
        print(f"form={form} n={n}: gen {gen_ok} msm {got == exp} host-api {host_api == exp}", flush=True)
# edge cases through the host API
cases = {
    "zeros": ([0] * 50, b.gen_bases(b.SEED_BASES, 50)),
    "ones": ([1] * 50, b.gen_bases(b.SEED_BASES, 50)),
    "r-1": ([b.R - 1] * 5, b.gen_bases(b.SEED_BASES, 5)),
    "repeated base": (b.gen_scalars(7, 40), [b.G1_GEN] * 40),
    "P,-P": ([5, 5, 9], [b.G1_GEN, b.g1_neg(b.G1_GEN), b.G1_GEN]),
    "identity bases": ([3, 4, 5], [None, b.G1_GEN, None]),
    "same scalar": ([123456789] * 200, b.gen_bases(b.SEED_BASES, 200)),
    "pow2": ([1 << k for k in range(254)], b.gen_bases(b.SEED_BASES, 254)),
}
for name, (sc, bs) in cases.items():
    got = svgpu.multi_scalar_multiplication(sc, bs)
    exp = b.native_msm(sc, bs)
    ok &= got == exp
    print(f"edge {name}: {got == exp}", flush=True)
# decider
g2, sg2, accs = b.gen_decider_case(6, bad=[3])
accs.append((None, None))
dk = svgpu.KzgDecidingKey(b.G1_GEN, g2, sg2)
lhs = torch.from_numpy(enc.bases_array([a[0] for a in accs]).view("int64")).to(dev)
rhs = torch.from_numpy(enc.bases_array([a[1] for a in accs]).view("int64")).to(dev)
t0 = time.time()
ff, verdicts, gts = dv.decide(g2, sg2, lhs, rhs, svgpu.SV_CANONICAL, want_gt=True)
print("decide first_fail", ff, verdicts, f"{time.time()-t0:.3f}s", flush=True)
exp_gt = [b.f12_to_list(b.decide_gt(g2, sg2, l, r)) for (l, r) in accs]
ok &= ff == 3 and gts == exp_gt
print("decider Gt parity", gts == exp_gt, flush=True)
print("host decide_all", svgpu.KzgAs.first_failure(dk, [svgpu.KzgAccumulator(*a) for a in accs]), flush=True)
# accumulate
acc2 = svgpu.KzgAs.create_proof([svgpu.KzgAccumulator(*a) for a in accs[:5]], 0x1234567)
ea = b.accumulate(accs[:5], 0x1234567)
ok &= (acc2.lhs, acc2.rhs) == ea
print("accumulate parity", (acc2.lhs, acc2.rhs) == ea, flush=True)
# timing at 2^20
n = 1 << 20
B = dv.gen_bases(dv.empty_bases(n, dev), b.SEED_BASES, 0, svgpu.SV_MONTGOMERY)
S = dv.gen_scalars(dv.empty_scalars(n, dev), b.SEED_SCALARS, 0, svgpu.SV_MONTGOMERY)
torch.cuda.synchronize()
for it in range(4):
    t0 = time.time(); r = dv.msm(B, S); t1 = time.time()
    print(f"2^20 msm {1000*(t1-t0):.2f} ms", dv.last_msm_stats(), flush=True)
# decider timing 256
g2, sg2, accs = b.gen_decider_case(16)
accs = accs * 16
lhs = torch.from_numpy(enc.bases_array([a[0] for a in accs]).view("int64")).to(dev)
rhs = torch.from_numpy(enc.bases_array([a[1] for a in accs]).view("int64")).to(dev)
for it in range(3):
    torch.cuda.synchronize(); t0 = time.time()
    ff, _, _ = dv.decide(g2, sg2, lhs, rhs)
    print(f"decide 256: ff={ff} {1000*(time.time()-t0):.2f} ms", flush=True)
print("ALL OK" if ok else "FAILURES", flush=True)
