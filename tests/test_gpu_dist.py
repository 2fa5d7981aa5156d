"""Two ranks on the GPU (gloo for the exchange, both processes on cuda:0): the point-sharded MSM
with the REAL per-rank device step (sv_bn254_g1_msm_device on each rank's HBM-resident shard) and
the accumulator-sharded decider with its MIN all-reduce, against the C++ oracle.  This is the
bench's N > 1 code path (svgpu.parallel) with nothing substituted; RCCL replaces gloo on a node.
The same path also runs over the nccl backend (RCCL) with one rank -- the one-GPU box cannot hold two
RCCL ranks (one rank per device) -- so the all-gather of the 96-B partials and the MIN all-reduce
go through RCCL on the device tensors exactly as in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, dn, bad, q, backend="gloo"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "snark-verifier-axiom_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    import svgpu
    from oracle import bn254 as b
    from svgpu import device as dv, encoding as enc, parallel
    svgpu.init()
    dev = torch.device("cuda:0")
    lo, hi = parallel.shard_range(n, rank, world)
    B = dv.gen_bases(dv.empty_bases(hi - lo, dev), b.SEED_BASES, lo, svgpu.SV_MONTGOMERY)
    S = dv.gen_scalars(dv.empty_scalars(hi - lo, dev), b.SEED_SCALARS, lo, svgpu.SV_MONTGOMERY)
    res = parallel.sharded_msm_device(B, S, svgpu.SV_MONTGOMERY)
    g2, sg2, accs = b.gen_decider_case(world * dn, seed=0xD15, bad=bad)
    mine = accs[rank * dn:(rank + 1) * dn]
    L = torch.from_numpy(enc.bases_array([a[0] for a in mine]).view(np.int64)).to(dev)
    R = torch.from_numpy(enc.bases_array([a[1] for a in mine]).view(np.int64)).to(dev)
    ff = parallel.sharded_decide_device(g2, sg2, L, R, rank * dn, svgpu.SV_CANONICAL)
    q.put((rank, res, ff, dist.get_backend()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("bad", [[], [37, 5], [3]])
def test_two_ranks_on_gpu_msm_and_decider(gpu, oracle_cpp, bad):
    from oracle import bn254 as b
    n, dn, world = 50001, 24, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, dn, bad, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    full = b.g1_from_bytes(oracle_cpp.msm_pippenger(B, S, 0).tobytes())
    assert out[0][1] == out[1][1] == full
    exp_ff = min(bad) if bad else -1
    assert out[0][2] == out[1][2] == exp_ff


@pytest.mark.timeout(300)
def test_rccl_single_rank_exchange(gpu, oracle_cpp):
    """svgpu.parallel over the nccl backend (RCCL): all_gather_into_tensor of the Jacobian partial
    and the MIN all-reduce of the first failing index on device tensors, one rank on cuda:0."""
    from oracle import bn254 as b
    n, dn, bad = 30011, 40, [29, 11]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), n, dn, bad, q, "nccl"))
    p.start()
    rank, res, ff, backend = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    B = oracle_cpp.gen_bases(b.SEED_BASES, n)
    S = oracle_cpp.gen_scalars(b.SEED_SCALARS, n)
    assert res == b.g1_from_bytes(oracle_cpp.msm_pippenger(B, S, 0).tobytes())
    assert ff == min(bad)
