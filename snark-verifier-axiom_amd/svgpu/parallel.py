"""Point-sharded MSM and accumulator-sharded decider across ranks (one process per GPU).

The reference is single-process; this is the build's multi-GPU layer:

* MSM: sum_i s_i P_i is additive over any partition.  Each rank reduces its contiguous shard to one
  Jacobian partial (96 B, canonical) with ``sv_bn254_g1_msm_device``; the exchange is ONE all-gather
  of those 96-byte records (RCCL over xGMI with the ``nccl`` backend; RCCL has no elliptic-curve
  reduction op, so all-gather + a fixed rank-order fold IS the all-reduce); every rank then folds
  the world's partials in rank order with ``sv_bn254_g1_fold``, so all ranks return the same point.
* Decider: accumulators are independent; each rank decides its shard and the first failing global
  index is combined with one ``MIN`` all-reduce (world size = "no failure").

``partial_fn`` lets CPU tests (gloo) substitute the per-rank device step; the exchange and fold
code is the production code either way.
"""
from __future__ import annotations

import struct
from typing import Callable, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .loader import Point, fold_partials

Jacobian = Tuple[int, int, int]


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    per = (n + world - 1) // world
    lo = min(n, rank * per)
    return lo, min(n, lo + per)


def _pack(j: Jacobian) -> np.ndarray:
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in j), dtype=np.uint8).copy()


def _unpack(buf: np.ndarray) -> Jacobian:
    raw = buf.tobytes()
    return tuple(int.from_bytes(raw[32 * k:32 * (k + 1)], "little") for k in range(3))  # type: ignore


def _comm_device(group) -> torch.device:
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def allgather_partials(partial: Jacobian, group=None) -> list:
    """All-gather one 96-byte Jacobian record per rank (rank order)."""
    world = dist.get_world_size(group)
    dev = _comm_device(group)
    mine = torch.from_numpy(_pack(partial)).to(dev)
    out = torch.empty(world * 96, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(out, mine, group=group)
    host = out.cpu().numpy()
    return [_unpack(host[96 * r:96 * (r + 1)]) for r in range(world)]


IDENTITY: Jacobian = (1, 1, 0)


def sharded_msm(partial_fn: Callable[[], Jacobian], group=None, local_terms: Optional[int] = None) -> Point:
    """Run this rank's shard (``partial_fn``), exchange partials, fold in rank order.  A rank whose
    shard is empty (``local_terms == 0``: more ranks than points, the tail of an uneven split)
    contributes the identity without calling ``partial_fn`` -- the library rejects an empty MSM --
    and still takes part in the all-gather."""
    partial = IDENTITY if local_terms == 0 else partial_fn()
    return fold_partials(allgather_partials(partial, group))


def sharded_msm_device(bases: torch.Tensor, scalars: torch.Tensor, form: int, group=None) -> Point:
    """``bases``/``scalars`` are THIS rank's shard, resident in HBM (possibly empty)."""
    from .device import msm_partial

    return sharded_msm(lambda: msm_partial(bases, scalars, form), group, local_terms=int(bases.shape[0]))


def combine_first_fail(local_first_fail: int, shard_offset: int, group=None) -> int:
    """Global first failing index from each rank's local one (-1 = none)."""
    world_sentinel = np.iinfo(np.int64).max
    dev = _comm_device(group)
    v = world_sentinel if local_first_fail < 0 else shard_offset + local_first_fail
    t = torch.tensor([v], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    g = int(t.item())
    return -1 if g == world_sentinel else g


def sharded_decide_device(g2, s_g2, lhs: torch.Tensor, rhs: torch.Tensor, shard_offset: int, form: int,
                          group=None) -> int:
    """decide_all over accumulator shards: this rank decides its HBM-resident shard (global indices
    [shard_offset, shard_offset + len)) and the first failing GLOBAL index (-1: all pass) comes
    from one MIN all-reduce, as the reference's sequential try_collect would report it
    (decider.rs:70-80)."""
    from .device import decide

    return sharded_decide(lambda: decide(g2, s_g2, lhs, rhs, form)[0], int(lhs.shape[0]), shard_offset, group)


def sharded_decide(local_fn: Callable[[], int], local_count: int, shard_offset: int, group=None) -> int:
    """The exchange of ``sharded_decide_device`` around any per-rank decider ``local_fn`` (local first
    failing index or -1).  An empty shard passes without a call (the library rejects an empty batch)
    and still joins the all-reduce."""
    local = -1 if local_count == 0 else local_fn()
    return combine_first_fail(local, shard_offset, group)
