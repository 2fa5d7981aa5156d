#!/usr/bin/env python3
"""bench.py -- BN254 G1 MSM points/s (headline) + KZG decider pairings/s on MI355X.

Metric (BASELINE.json): "BN254 G1 MSM points/sec at 2^20 + KZG pairings/sec; 1/2/4/8 GPU".
A "step" is one full MSM over the job's points, inputs already resident in HBM:
  N = 1: one 2^20-point MSM (config 2).
  N > 1: one MSM of N * 2^20 points, point-sharded (rank r holds points [r*2^20, (r+1)*2^20)),
         per-rank Pippenger on its GPU + ONE RCCL all-gather of the 96-byte Jacobian partials +
         rank-order fold on every rank (weak scaling: per-GPU work fixed).
`value` = total points / (max-over-ranks time of K steps).  Secondary: the KZG decider over 256
accumulators per GPU (config 3), pairings/s = 2 * accumulators / time.
CPU baseline (rank 0, N = 1): the C++ restatement of util::msm::multi_scalar_multiplication
(oracle/, "kind": "port") on the SAME 2^20 input with the host's threads, plus the sequential
decide_all on a 32-accumulator sample; the GPU result is checked against it (parity field).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]   (torchrun for N > 1)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X spec (MI355X_MICROARCH.md)
# v_mad_u64_u32 issue peak: one wave instruction per 4 clocks per SIMD (16 lanes / clk) x 4 SIMDs x 256
# CUs x 2.4 GHz = 64 lane-mads / clk / CU.  tools/ubench_issue.hip (round 5) measured 4.25 clocks per
# mad with 16 independent chains at 4 waves / SIMD (60.2 / clk / CU) and showed that every other VALU
# instruction takes issue time of its own (2-3.8 clocks): the bucket chain is bound by VALU issue, of
# which its mads are ~55 %.  (Rounds 1-4 used 32 / clk / CU, which the kernel appeared to exceed.)
MAC_PEAK = 64 * 256 * 2.4e9
MAC_PEAK_MEASURED = 64 * 4 / 4.25 * 256 * 2.4e9
MACS_PER_FPMUL = 136             # 8-limb CIOS: 64 + 64 + 8
# v_mad_u64_u32 per bucket entry that k_accumulate<false, true, 1> (the 29-bit chain) issues on its
# common path (no segment end, no doubling, no cancellation): r29::madd_live's nine field products --
# mul_sub<8> and five mul at 81 + 81, the square and sqr_sub2c<6> at 45 + 81, the fused Y3 pair
# mul_sum2 at 243 -- = 1467 (round 6; rounds 4-5's madd issued 1503).  The compiled loop's common
# blocks hold 1482 (tools/isa_count.py), the other 15 being address arithmetic.
MADS_PER_ENTRY_R29 = 1467
BYTES_PER_POINT = 96             # 64 B affine base + 32 B scalar, read once
# Decider algorithmic work: Fq products of ONE decide, COUNTED by instrumenting the C++
# restatements (oracle/cpu/bn254_ref.cpp; both pinned by tests/test_oracle_cpp.py):
#  * FPMUL_H2C_COUNTED -- the halo2curves-structured restatement (namespace h2c: Karatsuba towers,
#    complex and Granger-Scott cyclotomic squarings, sparse 034 lines, exp_by_x and the Scott et al.
#    hard part, G2 lines prepared inside every decide as decider.rs:64 does), i.e. the reference's
#    own work; its Gt value equals the plain restatement's.  The roofline's denominator.
#  * FPMUL_RESTATEMENT -- the plain restatement (dense line products, square-and-multiply final
#    exponentiation): an upper bound, reported for comparison.
FPMUL_H2C_COUNTED = 24710
FPMUL_RESTATEMENT = 57538
# of FPMUL_H2C_COUNTED, the two G2 line preparations (G2Prepared::from inside every decide,
# decider.rs:64), which the GPU decider caches per deciding key (or_count_h2c_prepare)
FPMUL_H2C_LINE_PREP = 5366


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--log-n", type=int, default=20, help="points per GPU = 2^log_n")
    ap.add_argument("--decider-n", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the batch-MSM / config-5 / Poseidon lines")
    ap.add_argument("--config4-log-n", type=int, default=24, help="one 2^k MSM split over the ranks (0: skip)")
    return ap.parse_args()


def ref_window(n: int) -> int:
    import math
    return int(math.ceil(math.log(n))) + 2


def _time(fn, reps):
    """Median over reps of one synchronised call (latency of the secondary rows; a single host-pool
    or clock hiccup would otherwise dominate a mean over 5 calls)."""
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)), r


CROSSOVER_SIZES = (1, 2, 3, 4, 8, 16, 32, 64)


def verifier_msm_rows(ob):
    """The native verifier's own MSMs: a handful of tens-term MSMs per proof (bdfg21.rs:75-78,
    gwc19.rs:76-79, reached from snark-verifier-sdk/src/halo2/aggregation.rs:219-233), each one
    NativeLoader::multi_scalar_multiplication call (native.rs:61-71).  (1) The crossover: one
    reference-shaped library call (sv_bn254_g1_msm_refs, host references, gather + transfer + the
    small-MSM window path) against the reference's naive sum of scalar muls (the C++ restatement,
    one thread) per size.  (2) 128 MSMs of 30 terms through 128 sequential calls and through one
    host-array batch call (sv_bn254_g1_msm_batch), against the naive CPU path."""
    import svgpu
    from oracle import cpu_ref
    C = svgpu.SV_CANONICAL
    count, m = 128, 30
    hb = cpu_ref.gen_bases(ob.SEED_BASES, count * m, start=31337)
    hs = cpu_ref.gen_scalars(ob.SEED_SCALARS, count * m, start=31337)

    def refs_of(lo, hi):
        idx = np.arange(lo, hi, dtype=np.uint64)
        return svgpu.make_refs(hs.ctypes.data + 32 * idx, hb.ctypes.data + 64 * idx)

    def med(fn, reps):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)) * 1e3
    cross = []
    for k in CROSSOVER_SIZES:
        rk = refs_of(0, k)
        g_ms = med(lambda: svgpu.msm_refs(rk, C), 25)
        c_ms = med(lambda: cpu_ref.msm_naive(hb[:k], hs[:k]), 3)
        cross.append({"terms": k, "gpu_call_ms": g_ms, "cpu_naive_ms": c_ms})
    faster = [c["terms"] for c in cross if c["gpu_call_ms"] < c["cpu_naive_ms"]]
    refs = [refs_of(i * m, (i + 1) * m) for i in range(count)]
    seq_ms = med(lambda: [svgpu.msm_refs(r, C) for r in refs], 3)
    off = list(range(0, count * m + 1, m))
    batch_ms = med(lambda: svgpu.msm_batch_arrays(hb, hs, off, C), 5)
    batch8_ms = med(lambda: svgpu.msm_batch_arrays(hb[:8 * m], hs[:8 * m], off[:9], C), 10)
    t0 = time.perf_counter()
    exp = [ob.g1_from_bytes(cpu_ref.msm_naive(hb[i * m:(i + 1) * m], hs[i * m:(i + 1) * m]).tobytes())
           for i in range(count)]
    cpu_ms = (time.perf_counter() - t0) * 1e3
    same = (svgpu.msm_batch_arrays(hb, hs, off, C) == exp
            and [svgpu.msm_refs(r, C) for r in refs[:8]] == exp[:8])
    return {"crossover": cross, "gpu_faster_from_terms": min(faster) if faster else None,
            "msms": count, "terms_each": m, "sequential_calls_ms": seq_ms, "one_batch_call_ms": batch_ms,
            "batch_of_8_ms": batch8_ms, "cpu_naive_1_thread_ms": cpu_ms,
            "x_vs_cpu_sequential": cpu_ms / seq_ms, "x_vs_cpu_batch": cpu_ms / batch_ms,
            "parity_vs_oracle": bool(same),
            "note": "host arrays, canonical form; sequential = one sv_bn254_g1_msm_refs call per MSM (what the "
                    "Rust shim's NativeLoader routing issues); batch = sv_bn254_g1_msm_batch; CPU = the naive "
                    "NativeLoader restatement (one scalar mul + add per term) on one thread"}


def next_rows(dev, dv, ob, enc, g2, sg2, accs):
    import svgpu
    M = svgpu.SV_MONTGOMERY
    res = {}
    # f1: 128 MSMs x 64 terms (the per-proof pair of a 64-proof aggregation) in one launch
    count, m = 128, 64
    B = dv.gen_bases(dv.empty_bases(count * m, dev), ob.SEED_BASES, 0, M)
    S = dv.gen_scalars(dv.empty_scalars(count * m, dev), ob.SEED_SCALARS, 0, M)
    off = torch.arange(0, count * m + 1, m, dtype=torch.int64, device=dev)
    t, _ = _time(lambda: dv.msm_batch(B, S, off, m, M), 5)
    res["msm_batch"] = {"msms": count, "terms_each": m, "ms": t * 1e3, "terms_per_s": count * m / t}
    # a few proofs' MSMs (8 x 64 terms): the small-batch route, window sums on the device and the
    # Horners on the host (SVGPU_BATCH_HOST_MAX), against the fused kernel's one-wave chain
    small = {}
    for route, hm in (("host_horner", None), ("fused", "0")):
        old = os.environ.pop("SVGPU_BATCH_HOST_MAX", None)
        if hm is not None:
            os.environ["SVGPU_BATCH_HOST_MAX"] = hm
        ts, _ = _time(lambda: dv.msm_batch(B, S, off[:9], m, M), 5)
        small[route] = ts * 1e3
        os.environ.pop("SVGPU_BATCH_HOST_MAX", None)
        if old is not None:
            os.environ["SVGPU_BATCH_HOST_MAX"] = old
    same_small = bool(torch.equal(dv.msm_batch(B, S, off[:9], m, M), dv.msm_batch(B, S, off, m, M)[:8]))
    res["msm_batch_small"] = {"msms": 8, "terms_each": m, "ms": small["host_horner"], "fused_ms": small["fused"],
                              "same_result_as_fused_batch": same_small}
    res["verifier_msms"] = verifier_msm_rows(ob)
    # f1 with fixed bases: the same batch, each term referencing a row of a 4096-row base table
    #   (created once, rows precomputed as 2^(8w) P: one bucket set per MSM, no window Horner)
    rows = 4096
    Th = dv.gen_bases(dv.empty_bases(rows, dev), ob.SEED_BASES, 0, svgpu.SV_CANONICAL).cpu().numpy().view(np.uint64)
    t0 = time.perf_counter()
    tab = svgpu.BaseTable(Th)
    create_ms = (time.perf_counter() - t0) * 1e3
    idx = torch.randint(0, rows, (count * m,), dtype=torch.int32, device=dev)
    t, _ = _time(lambda: tab.msm_batch_device(idx, S, off, M), 5)
    Tm = dv.gen_bases(dv.empty_bases(rows, dev), ob.SEED_BASES, 0, M)
    same = bool(torch.equal(tab.msm_batch_device(idx, S, off, M), dv.msm_batch(Tm[idx.long()].contiguous(), S, off, m, M)))
    tab.close()
    res["msm_batch_table"] = {"msms": count, "terms_each": m, "table_rows": rows, "ms": t * 1e3,
                              "terms_per_s": count * m / t, "table_create_ms": create_ms,
                              "same_result_as_plain_batch": same}
    # config 5: 64 valid accumulators -> KzgAs::create_proof (fresh Poseidon transcript absorbs every
    # lhs/rhs, squeezes r; MSMs with r^0..r^63) -> one decide (accumulation.rs:146-195, decider.rs:60-68)
    acc64 = accs[:64]
    inst = [svgpu.KzgAccumulator(a[0], a[1]) for a in acc64]
    dk = svgpu.KzgDecidingKey(ob.G1_GEN, g2, sg2)

    def aggregate():
        acc = svgpu.KzgAs.create_proof(inst, svgpu.PoseidonTranscript())
        svgpu.KzgAs.decide(dk, acc)
        return acc
    t, acc = _time(aggregate, 5)
    (el, er), r_exp, _ = ob.create_proof(acc64)
    parity = bool((acc.lhs, acc.rhs) == (el, er) and svgpu.KzgAs.last_challenge == r_exp)
    t_acc, _ = _time(lambda: svgpu.KzgAs.create_proof(inst, r_exp), 5)
    res["config5_aggregation"] = {"accumulators": 64, "latency_ms": t * 1e3, "verdict": "pass",
                                  "challenge": "poseidon transcript (host sponge)",
                                  "accumulate_given_r_ms": t_acc * 1e3, "parity_vs_oracle": parity}
    # f2: batched Poseidon permutations (t = 3, the SDK transcript's width), HBM-resident states
    n = 1 << 20
    st = torch.randint(0, 1 << 62, (n * 3, 4), dtype=torch.int64, device=dev)
    st[:, 3] &= (1 << 59) - 1
    t, _ = _time(lambda: dv.poseidon_permute(st, 3, M), 5)
    res["poseidon"] = {"width": 3, "states": n, "ms": t * 1e3, "permutations_per_s": n / t}
    return res


def affinity_cores() -> int:
    """Cores this process may run on (sched_getaffinity): what rayon's default pool would use for
    the reference's `parallel` Pippenger (util.rs:83-152, msm.rs:290-310)."""
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)


def cpu_threads() -> int:
    """Host threads for the CPU legs: every core this process may run on, capped by the box's
    OMP_NUM_THREADS share when that is set (one GPU's slice of a shared node)."""
    cores = affinity_cores()
    share = os.environ.get("OMP_NUM_THREADS")
    return min(cores, int(share)) if share and share.isdigit() and int(share) > 0 else cores


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, n, gpu_result, g2, sg2, accs, enc):
    """The reference's CPU paths, restated in C++ (oracle/, "kind": "port"), timed on this host:
    a3 Pippenger on all allowed threads (msm.rs:238-316 with `parallel`), a1 NativeLoader's naive
    sum of scalar muls on one thread (native.rs:61-71) at 2^10 / 2^12 with its linear scaling,
    a8 decide_all sequential (decider.rs:70-80) and an all-cores upper bound, and config 5
    (accumulate 64 accumulators with naive MSMs, accumulation.rs:146-195, then one decide)."""
    from oracle import bn254 as ob
    from oracle import cpu_ref
    threads = cpu_threads()
    hb = cpu_ref.gen_bases(ob.SEED_BASES, n, threads=threads)
    hs = cpu_ref.gen_scalars(ob.SEED_SCALARS, n)
    t0 = time.perf_counter()
    cpu_res = cpu_ref.msm_pippenger(hb, hs, threads)
    cpu_s = time.perf_counter() - t0
    parity = ob.g1_from_bytes(cpu_res.tobytes()) == gpu_result
    # the same port on every core the affinity mask allows (rayon's default would take them all)
    aff_cores = affinity_cores()
    aff_s = None
    if aff_cores != threads:
        t0 = time.perf_counter()
        aff_res = cpu_ref.msm_pippenger(hb, hs, aff_cores)
        aff_s = time.perf_counter() - t0
        parity = parity and ob.g1_from_bytes(aff_res.tobytes()) == gpu_result
    naive = {}
    for lg in (10, 12):
        m = 1 << lg
        t0 = time.perf_counter()
        cpu_ref.msm_naive(hb[:m], hs[:m])
        naive["2^%d_seconds" % lg] = time.perf_counter() - t0
    naive_pps = (1 << 12) / naive["2^12_seconds"]
    g2b = np.frombuffer(ob.g2_bytes(g2), np.uint64)
    sg2b = np.frombuffer(ob.g2_bytes(sg2), np.uint64)
    ds = 32
    dL = enc.bases_array([a[0] for a in accs[:ds]])
    dR = enc.bases_array([a[1] for a in accs[:ds]])
    t0 = time.perf_counter()
    cff, _ = cpu_ref.decide_all(g2b, sg2b, dL, dR, threads=1)
    cdec = time.perf_counter() - t0
    aL = enc.bases_array([a[0] for a in accs])
    aR = enc.bases_array([a[1] for a in accs])
    t0 = time.perf_counter()
    aff, _ = cpu_ref.decide_all(g2b, sg2b, aL, aR, threads=threads)
    adec = time.perf_counter() - t0
    r = ob.gen_scalar(ob.SEED_SCALARS, 1 << 30)
    rr = np.array([(r >> (64 * k)) & ((1 << 64) - 1) for k in range(4)], np.uint64)
    t0 = time.perf_counter()
    ol, orr = cpu_ref.accumulate(aL[:64], aR[:64], rr)
    c5ff, _ = cpu_ref.decide_all(g2b, sg2b, ol.reshape(1, 8), orr.reshape(1, 8), threads=1)
    c5 = time.perf_counter() - t0
    return {
        "value": n / cpu_s,
        "unit": "points/s",
        "cores": threads,
        "kind": "port",
        "sample": "the same 2^%d-point MSM, C++ restatement of util::msm::multi_scalar_multiplication "
                  "(msm.rs:238-316: window ceil(ln n)+2, one chunk per thread) on %d host threads; "
                  "naive NativeLoader MSM (native.rs:61-71) on 1 thread at 2^10 and 2^12; decide_all over %d "
                  "accumulators on 1 thread (decider.rs:70-80 is sequential) and over %d on %d threads; "
                  "config 5: accumulate 64 + one decide on 1 thread" % (args.log_n, threads, ds, len(accs), threads),
        "cpu_model": cpu_model(),
        "host_cpus_visible": os.cpu_count(),
        "affinity_cores": aff_cores,
        "threads_note": "cores = min(affinity cores, OMP_NUM_THREADS share of this GPU's box slice); "
                        "value_affinity_cores runs one thread per affinity core, which the box's cgroup CPU "
                        "quota (cpu.max 1600000/100000 = 16 CPUs) throttles below the 16-thread value",
        "value_affinity_cores": n / aff_s if aff_s else n / cpu_s,
        "seconds": cpu_s,
        "parity_vs_gpu": bool(parity and cff == -1 and aff == -1 and c5ff == -1),
        "naive_nativeloader": {
            **naive,
            "points_per_s_1_thread": naive_pps,
            "scaling": "linear in n (one ~256-bit double-and-add per pair): t(n) = n / points_per_s",
            "extrapolated_2^20_seconds": (1 << 20) / naive_pps,
        },
        "kzg_pairings_per_s": 2 * ds / cdec,
        "kzg_pairings_per_s_all_cores": 2 * len(accs) / adec,
        "config5_latency_ms_1_thread": c5 * 1e3,
    }


SETTLE_STEPS = 30


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one process per GPU; SVGPU_DIST_BACKEND=gloo lets several ranks share one card (rehearsal)
    backend = os.environ.get("SVGPU_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    local_dev = local % ndev if backend == "gloo" else local
    torch.cuda.set_device(local_dev)
    dev = torch.device("cuda", local_dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")

    import svgpu
    from svgpu import device as dv, parallel
    from oracle import bn254 as ob

    svgpu.init()
    n = 1 << args.log_n
    form = svgpu.SV_MONTGOMERY  # halo2curves' in-memory layout (zero-copy from Rust)
    B = dv.gen_bases(dv.empty_bases(n, dev), ob.SEED_BASES, rank * n, form)
    S = dv.gen_scalars(dv.empty_scalars(n, dev), ob.SEED_SCALARS, rank * n, form)
    torch.cuda.synchronize()

    def step():
        if world > 1:
            return parallel.sharded_msm_device(B, S, form)
        return dv.msm(B, S, form)

    def barrier():
        if world > 1:
            dist.barrier()

    # the first ~5 back-to-back steps after start-up run ~4 % slow while the GPU settles
    # (tools/step_jitter.py: 2.05 -> 1.96 ms); settle on untimed steps before the W warmup steps
    for _ in range(SETTLE_STEPS):
        step()
    for _ in range(args.warmup):
        result = step()
    barrier()
    torch.cuda.synchronize()
    acc_ms, span_ms = [], []
    # timed steps record only the accumulate's two HIP events (the live roofline); the sort /
    # reduce split costs two more event records per call and is taken from one step afterwards
    os.environ["SVGPU_MSM_LEAN"] = "1"
    t0 = time.perf_counter()
    for _ in range(args.steps):
        result = step()
        st_ = dv.last_msm_stats()
        acc_ms.append(st_["accumulate_ms"])
        span_ms.append(st_["accumulate_span_ms"])
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    os.environ["SVGPU_MSM_LEAN"] = "0"
    step()
    torch.cuda.synchronize()
    stats = dv.last_msm_stats()
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    total_points = n * world
    value = total_points * args.steps / elapsed

    # ---- the host-buffer entry points the Rust shim binds, same 2^log_n input:
    #      sv_bn254_g1_msm from pageable Montgomery arrays (halo2curves' layout, zero-copy from
    #      Rust; the H2D transfer is inside the timing) and sv_bn254_g1_msm_refs over shuffled
    #      references (NativeLoader's &[(&Fr, &G1Affine)] shape: the gather is inside too)
    host_api = None
    if rank == 0 and world == 1 and not args.no_extras:
        hB = B.cpu().numpy().view(np.uint64).copy()
        hS = S.cpu().numpy().view(np.uint64).copy()

        def med(fn, reps=7):
            fn()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                r = fn()
                ts.append(time.perf_counter() - t0)
            return float(np.median(ts)), r
        h_s, h_res = med(lambda: svgpu.msm_arrays(hB, hS, form))
        perm = np.random.default_rng(7).permutation(n)
        refs = svgpu.make_refs(hS.ctypes.data + 32 * perm.astype(np.uint64), hB.ctypes.data + 64 * perm.astype(np.uint64))
        r_s, r_res = med(lambda: svgpu.msm_refs(refs, form))
        dev_ms = elapsed / args.steps * 1e3
        host_api = {
            "msm_host_ms": h_s * 1e3,
            "msm_host_points_per_s": n / h_s,
            "x_device_resident": h_s * 1e3 / dev_ms,
            "refs_gather_inclusive_ms": r_s * 1e3,
            "refs_x_device_resident": r_s * 1e3 / dev_ms,
            "h2d_pieces": os.environ.get("SVGPU_H2D_PIECES", os.environ.get(
                "SVGPU_H2D_SPLIT", "default: 5,4,4,3 (msm), 2,2,3,3,3,3 (refs)")),
            "same_result_as_device_path": bool(h_res == result and r_res == result),
            "note": "sv_bn254_g1_msm: pageable host arrays -> HBM in pieces, staged back to back by the workspace's "
                    "feeder thread; each piece sorted on a second stream once its scalars land and accumulated into "
                    "the one bucket set once its bases land (median of 7 calls, transfer included); "
                    "sv_bn254_g1_msm_refs: 2^%d shuffled (&Fr, &G1Affine) references gathered by the library's "
                    "host pool into pinned staging, piece by piece (gather + transfer included)" % args.log_n,
        }
        del hB, hS, refs

    # ---- KZG decider (config 3): accumulators per GPU (N > 1: rank r holds global accumulators
    #      [r dn, (r + 1) dn) and the first failing global index comes from one MIN all-reduce)
    dn = args.decider_n
    # dn distinct valid accumulators per rank (rank r: the seeded t_i for i in [r dn, (r + 1) dn))
    g2, sg2, accs = ob.gen_decider_case(dn, seed=ob.SEED_TRAPDOOR, start=rank * dn)
    from svgpu import encoding as enc
    L = torch.from_numpy(enc.bases_array([a[0] for a in accs]).view(np.int64)).to(dev)
    R = torch.from_numpy(enc.bases_array([a[1] for a in accs]).view(np.int64)).to(dev)

    def decide_step():
        if world > 1:
            return parallel.sharded_decide_device(g2, sg2, L, R, rank * dn, svgpu.SV_CANONICAL)
        ff_, _, _ = dv.decide(g2, sg2, L, R)
        return ff_
    # the decider line's own loop: a call is ~0.5 ms, so a few warm calls and at least 20 timed ones
    # (5 right after one call read 0.56 ms per call on a box whose steady state was 0.52)
    dwarm = max(3, args.warmup)
    for _ in range(dwarm):
        ff = decide_step()
    dsteps = max(20, 2 * args.steps)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dec_kernel_ms = []
    for _ in range(dsteps):
        ff = decide_step()
        dec_kernel_ms.append(dv.last_decide_kernel_ms())
    torch.cuda.synchronize()
    barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dec_s = float(dt.item())
    pairings_per_s = 2 * dn * world * dsteps / dec_s

    # ---- config 4: ONE 2^24-point MSM split over the N ranks (strong scaling; the north-star
    #      target is >= 1e8 scalar-muls/s at N = 8), inputs generated in each rank's HBM
    c4 = None
    if args.config4_log_n > 0:
        del B, S
        torch.cuda.empty_cache()
        n4 = (1 << args.config4_log_n) // world
        B4 = dv.gen_bases(dv.empty_bases(n4, dev), ob.SEED_BASES, rank * n4, form)
        S4 = dv.gen_scalars(dv.empty_scalars(n4, dev), ob.SEED_SCALARS, rank * n4, form)
        torch.cuda.synchronize()

        def step4():
            if world > 1:
                return parallel.sharded_msm_device(B4, S4, form)
            return dv.msm(B4, S4, form)
        res4 = step4()
        c4steps = max(1, args.steps // 5)
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(c4steps):
            step4()
        torch.cuda.synchronize()
        barrier()
        t4 = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t4, op=dist.ReduceOp.MAX)
        t4 = float(t4.item()) / c4steps
        c4 = {"points": n4 * world, "points_per_gpu": n4, "ms_per_msm": t4 * 1e3,
              "scalar_muls_per_s": n4 * world / t4, "scaling": "strong (fixed 2^%d total)" % args.config4_log_n,
              "north_star_target_at_8_gpus": 1e8}
        del B4, S4
        torch.cuda.empty_cache()
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            # parity at the config-4 size: the same 2^k MSM (canonical copy of the same seeded
            # points) through the C++ restatement of msm.rs:238-316 on the host cores
            from oracle import cpu_ref
            Bc = dv.gen_bases(dv.empty_bases(n4, dev), ob.SEED_BASES, 0, svgpu.SV_CANONICAL)
            Sc = dv.gen_scalars(dv.empty_scalars(n4, dev), ob.SEED_SCALARS, 0, svgpu.SV_CANONICAL)
            hb4 = Bc.cpu().numpy().view(np.uint64)
            hs4 = Sc.cpu().numpy().view(np.uint64)
            del Bc, Sc
            torch.cuda.empty_cache()
            t0 = time.perf_counter()
            exp4 = ob.g1_from_bytes(cpu_ref.msm_pippenger(hb4, hs4, cpu_threads()).tobytes())
            c4["oracle_seconds"] = time.perf_counter() - t0
            c4["parity_vs_oracle"] = bool(exp4 == res4)
            del hb4, hs4

    # ---- "next" rows, rank 0 only: batched small MSMs, config-5 aggregation
    #      latency (accumulate 64 accumulators with r^i, then decide), batched Poseidon permutations
    extra = {}
    if rank == 0 and not args.no_extras:
        extra = next_rows(dev, dv, ob, enc, g2, sg2, accs)

    # ---- roofline of the dominant kernel (k_accumulate), timed with HIP events on its stream
    # k_accumulate launches per MSM: 2 when the window halves run as separate launches (the second
    # beside the first half's reduction); accumulate_ms sums the launches' own durations,
    # accumulate_span_ms runs from the first launch's start to the last one's end
    groups = int(stats.get("accumulate_launches", 1)) or 1
    acc_sum_ms = float(np.mean(acc_ms))
    acc_span_ms = float(np.mean(span_ms))
    acc_avg_ms = acc_sum_ms / groups
    entries = stats["entries"]
    bytes_per_launch = BYTES_PER_POINT * n / groups
    ach_gbs = bytes_per_launch / (acc_avg_ms * 1e-3) / 1e9
    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_accumulate.json")
    if os.path.exists(prof):
        try:
            traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    macs = entries * 10 * MACS_PER_FPMUL  # one mixed XYZZ add (8M + 2S) per bucket entry, 8x32-bit work
    issued = entries * MADS_PER_ENTRY_R29  # what the 29-bit chain issues
    # VALU issue of k_accumulate from the round's SQ pass (profiles/*_sq_counters.json): wave
    # instructions per dispatch x 4 clocks over the launch's SIMD-clocks (live kernel time)
    valu = None
    sqf = sorted(f for f in os.listdir(os.path.join(ROOT, "profiles")) if f.endswith("_sq_counters.json"))
    try:  # the SQ pass of the same evidence run as profiles/pmc_accumulate.json (its "source" tag)
        tag = os.path.basename(json.load(open(os.path.join(ROOT, "profiles", "pmc_accumulate.json")))["source"])
        tag = tag.replace("_kernel_stats.md", "_sq_counters.json")
        if tag in sqf:
            sqf.append(tag)
    except (OSError, KeyError, ValueError):
        pass
    if sqf:
        try:
            sqd = json.load(open(os.path.join(ROOT, "profiles", sqf[-1])))
            ka = next(v for k, v in sqd.items() if k.startswith("k_accumulate") and "SQ_INSTS_VALU" in v)
            vi = ka["SQ_INSTS_VALU"]
            valu = {"source": "profiles/" + sqf[-1], "valu_wave_insts_per_dispatch": vi,
                    "valu_per_entry_wave": vi / (entries / 64.0),
                    "int64_share": ka.get("SQ_INSTS_VALU_INT64", 0) / vi if vi else None,
                    "issue_frac_4clk": vi * 4 / (acc_avg_ms * 1e-3 * 2.4e9 * 1024)}
        except (StopIteration, KeyError, ValueError, OSError):
            valu = None
    c_ref = ref_window(n)
    W_ref = -(-256 // c_ref)
    ref_macs = (W_ref * n * 11 + W_ref * 2 * ((1 << c_ref) - 1) * 16) * MACS_PER_FPMUL

    out = {
        "metric": "BN254 G1 MSM points/sec at 2^20 + KZG pairings/sec; 1/2/4/8 GPU",
        "value": value,
        "unit": "points/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_steps": SETTLE_STEPS,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (254-bit Montgomery field: bucket chain 9x29-bit limbs, elsewhere 8x32-bit)",
        "data": "synthetic (SplitMix64 seeded scalars < r, try-and-increment points on y^2=x^3+3)",
        "config": {
            "workload": "BN254 G1 Pippenger MSM, 2^%d random points/scalars per GPU (config 2 at N=1; "
                        "N>1: one %d-point MSM point-sharded with an RCCL all-gather of Jacobian partials)"
                        % (args.log_n, total_points),
            "points_per_gpu": n,
            "total_points": total_points,
            "input_form": "montgomery (halo2curves layout), HBM-resident",
            "window_bits": stats["window_bits"],
            "windows": stats["num_windows"],
            "parallelism": "point-sharded x%d" % world,
            "dist": ({"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                      "exchange": "all_gather_into_tensor of 96-B Jacobian partials + rank-order fold; "
                                  "decider: MIN all-reduce of first_fail"}
                     if world > 1 else {"backend": None, "world_size": 1}),
        },
        "kzg": {
            "pairings_per_s": pairings_per_s,
            "checks_per_s": pairings_per_s / 2,
            "accumulators_per_gpu": dn,
            "ms_per_decide_all": dec_s / dsteps * 1e3,
            "calls": {"warmup": dwarm, "timed": dsteps},
            "kernel_ms": float(np.mean(dec_kernel_ms)),
            "first_fail": ff,
            "fpmul_per_check": {"h2c_restatement_counted": FPMUL_H2C_COUNTED,
                                "plain_restatement_counted": FPMUL_RESTATEMENT},
            "int_mac": {
                "achieved": dn * FPMUL_H2C_COUNTED * MACS_PER_FPMUL / (np.mean(dec_kernel_ms) * 1e-3),
                "frac": dn * FPMUL_H2C_COUNTED * MACS_PER_FPMUL / (np.mean(dec_kernel_ms) * 1e-3) / MAC_PEAK,
                "frac_without_line_prep": dn * (FPMUL_H2C_COUNTED - FPMUL_H2C_LINE_PREP) * MACS_PER_FPMUL
                                          / (np.mean(dec_kernel_ms) * 1e-3) / MAC_PEAK,
                "peak": MAC_PEAK,
                "unit": "MAC/s (v_mad_u64_u32), work = accumulators x h2c_restatement_counted Fq products x 136; "
                        "frac_without_line_prep drops the %d products of the two G2 line preparations the kernel "
                        "caches per key" % FPMUL_H2C_LINE_PREP,
            },
        },
        "breakdown_ms": {k: round(stats[k], 4) for k in
                         ("sort_ms", "accumulate_ms", "reduce_ms", "host_ms", "total_ms")},
        "breakdown_note": "HIP events on the library stream: sort_ms = digit extraction + two-level counting sort "
                          "(digits never stored; the GLV halves kept for the scatter pass), reduce_ms = bucket fixup + reduction, host_ms = host Horner; "
                          "finer splits with SVGPU_MSM_STATS=1 (each extra event costs ~5 us of GPU idle)",
        "roofline": {
            "bound": "hbm",
            "kernel": "k_accumulate",
            "achieved": ach_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": ach_gbs / HBM_PEAK_GBS,
            "traffic": traffic,
            "kernel_avg_ms": acc_avg_ms,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "launches_per_msm": groups,
            "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None,
            "note": "path is VALU-issue bound (integer multiply + carry handling), not HBM: see int_mac",
        },
        "int_mac": {
            "kernel_issued_mads_per_entry": MADS_PER_ENTRY_R29,
            "kernel_achieved": issued / (acc_span_ms * 1e-3),
            "kernel_frac": issued / (acc_span_ms * 1e-3) / MAC_PEAK,
            "kernel_frac_of_measured_peak": issued / (acc_span_ms * 1e-3) / MAC_PEAK_MEASURED,
            "equiv32_achieved": macs / (acc_span_ms * 1e-3),
            "equiv32_frac": macs / (acc_span_ms * 1e-3) / MAC_PEAK,
            "kernel_time": "accumulate span (first k_accumulate start to last end) %.4f ms; launches' own "
                           "durations sum to %.4f ms" % (acc_span_ms, acc_sum_ms),
            "msm_achieved_ref_work": ref_macs / (elapsed / args.steps),
            "msm_frac_ref_work": ref_macs / (elapsed / args.steps) / MAC_PEAK,
            "peak": MAC_PEAK,
            "peak_measured": MAC_PEAK_MEASURED,
            "valu_issue": valu,
            "unit": "MAC/s (v_mad_u64_u32).  kernel_*: the mads the 29-bit chain issues (tools/isa_count.py); "
                    "equiv32_*: the 8x32-bit work it replaces (10 products x 136 per entry); peak: one wave "
                    "mad per 4 clocks per SIMD, peak_measured: tools/ubench_issue.hip",
        },
    }

    if host_api is not None:
        out["host_api"] = host_api
    if c4 is not None:
        out["config4_msm_2_24"] = c4
    out.update(extra)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, n, result, g2, sg2, accs, enc)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
