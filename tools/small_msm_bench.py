"""Latency of one small host-buffer MSM (sv_bn254_g1_msm, canonical arrays already encoded) for
n = 16 ... 256 terms: the round-5 small-MSM path (k_batch_uwin + host Horner) and, with
SVGPU_SMALL_MSM=0 in the environment, the single pipeline.  Median of 50 calls after 5 warm-ups;
the first call per n is checked against the oracle."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd")); sys.path.insert(0, ROOT)
import svgpu
from svgpu import encoding as enc
from oracle import bn254 as ob
svgpu.init()
tag = "pipeline" if os.environ.get("SVGPU_SMALL_MSM") == "0" else "small-msm path"
for n in (16, 32, 64, 128, 256):
    scal, pts = ob.gen_scalars(1000 + n, n), ob.gen_bases(1000 + n, n)
    B, S = enc.bases_array(pts), enc.scalars_array(scal)
    got = svgpu.msm_arrays(B, S)
    assert got == ob.native_msm(scal, pts), n
    for _ in range(5):
        svgpu.msm_arrays(B, S)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter()
        svgpu.msm_arrays(B, S)
        ts.append(time.perf_counter() - t0)
    ts.sort()
    print(f"{tag}: n={n:4d}  median {ts[25]*1e3:.3f} ms  min {ts[0]*1e3:.3f} ms", flush=True)
