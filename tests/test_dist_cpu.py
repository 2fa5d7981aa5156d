"""World-size-2 gloo run of the sharded MSM / decider exchange (svgpu.parallel) on CPU.

The per-rank device step is substituted by the C++ oracle (test infrastructure); the shard
ranges, the 96-byte all-gather and the rank-order fold are the production code."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _jacobian_of_affine(row):
    from oracle import bn254 as b
    p = b.g1_from_bytes(row.tobytes())
    if p is None:
        return (1, 1, 0)
    z = 7  # any non-unit Z exercises the fold's projective path
    return (p[0] * z * z % b.P, p[1] * z**3 % b.P, z)


def _worker(rank, world, port, n, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import bn254 as b, cpu_ref
    from svgpu import parallel
    B = cpu_ref.gen_bases(b.SEED_BASES, n, threads=1)
    S = cpu_ref.gen_scalars(b.SEED_SCALARS, n)
    lo, hi = parallel.shard_range(n, rank, world)
    res = parallel.sharded_msm(lambda: _jacobian_of_affine(cpu_ref.msm_pippenger(B[lo:hi], S[lo:hi], 1)))
    ff = parallel.combine_first_fail(1 if rank == 1 else -1, lo)
    ff_none = parallel.combine_first_fail(-1, lo)
    q.put((rank, res, ff, ff_none, lo))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_msm_gloo_world2():
    from oracle import bn254 as b, cpu_ref
    n = 301
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = cpu_ref.gen_bases(b.SEED_BASES, n, threads=1)
    S = cpu_ref.gen_scalars(b.SEED_SCALARS, n)
    full = b.g1_from_bytes(cpu_ref.msm_pippenger(B, S, 1).tobytes())
    assert out[0][1] == out[1][1] == full
    lo1 = out[1][4]
    assert out[0][2] == out[1][2] == lo1 + 1
    assert out[0][3] == out[1][3] == -1


def test_shard_ranges_cover_exactly():
    from svgpu.parallel import shard_range
    for n in (1, 7, 8, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def _worker4(rank, world, port, cases, q):
    """World-size-4 exchange with uneven shards: per case, the MSM of n points and the decider over
    n accumulators (some failing), each rank running its own contiguous shard (possibly empty)."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import bn254 as b, cpu_ref
    from svgpu import encoding as enc, parallel
    out = []
    for n, bad in cases:
        B = cpu_ref.gen_bases(b.SEED_BASES, n, threads=1)
        S = cpu_ref.gen_scalars(b.SEED_SCALARS, n)
        lo, hi = parallel.shard_range(n, rank, world)
        calls = []

        def part():
            calls.append(hi - lo)
            return _jacobian_of_affine(cpu_ref.msm_pippenger(B[lo:hi], S[lo:hi], 1))
        res = parallel.sharded_msm(part, local_terms=hi - lo)
        g2, sg2, accs = b.gen_decider_case(n, seed=0x4444, bad=bad)
        L = enc.bases_array([a[0] for a in accs[lo:hi]])
        R = enc.bases_array([a[1] for a in accs[lo:hi]])
        G2, SG2 = np.frombuffer(b.g2_bytes(g2), np.uint64), np.frombuffer(b.g2_bytes(sg2), np.uint64)

        def local_decide():
            calls.append(-(hi - lo))
            return cpu_ref.decide_all(G2, SG2, L, R, threads=1)[0]
        ff = parallel.sharded_decide(local_decide, hi - lo, lo)
        out.append((lo, hi, res, ff, calls))
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_exchange_gloo_world4_uneven():
    """gloo world size 4: n not divisible by the world size, an empty last
    shard (no library call on it, identity partial, still in the collectives), and a failing
    accumulator in the last non-empty shard; every rank returns the whole MSM and the global first
    failure, as decide_all's sequential try_collect reports it (decider.rs:70-80)."""
    from oracle import bn254 as b, cpu_ref
    cases = [(13, [12]), (9, [7, 8]), (6, [])]   # shards 4,4,4,1 / 3,3,3,0 / 2,2,2,0
    world = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker4, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k, (n, bad) in enumerate(cases):
        B = cpu_ref.gen_bases(b.SEED_BASES, n, threads=1)
        S = cpu_ref.gen_scalars(b.SEED_SCALARS, n)
        full = b.g1_from_bytes(cpu_ref.msm_pippenger(B, S, 1).tobytes())
        exp_ff = min(bad) if bad else -1
        spans = []
        for r in range(world):
            lo, hi, res, ff, calls = got[r][k]
            spans.append((lo, hi))
            assert res == full, (n, r)
            assert ff == exp_ff, (n, r)
            assert calls == ([] if hi == lo else [hi - lo, -(hi - lo)]), (n, r)
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    assert got[3][1][0] == got[3][1][1] == 9  # case 2's last shard is empty
