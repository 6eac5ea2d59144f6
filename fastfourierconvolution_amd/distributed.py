"""Sample-sharded execution across the GPUs of one node (one process per GPU, RCCL over xGMI).

The FFC forward is per-sample except for train-mode BatchNorm: every layer
maps sample b to sample b, so a global batch split over ranks gives the global result as
long as the BN batch statistics are global.  That is the only exchange on the data path:

  * weights / buffers: ``broadcast_module`` once at init (rank 0's copy wins);
  * BN moments:        ``enable_sync_bn`` routes the per-channel fp64 raw moments
                       {count, sum x, sum x^2} of every train-mode BN (SpectralTransform.bn1,
                       FourierUnitSN.bn, FFC_BN_ACT bn_l/bn_g) through ``all_reduce(SUM)``
                       before scale/shift are formed (``merge_moments``), so the sharded
                       forward equals the global-batch forward and the running statistics
                       stay identical on every rank;
  * outputs:           ``gather_batch`` (all_gather) when a caller wants the global batch.

Nothing here moves activations between GPUs.  The reference has no multi-GPU path of its own
for this block (it trains on one device); this is the partitioning ``north_star`` asks for.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _runtime as rt

__all__ = ["shard_range", "shard_batch", "broadcast_module", "enable_sync_bn", "disable_sync_bn",
           "merge_moments", "gather_batch"]


def shard_range(global_batch: int, rank: int, world: int) -> tuple[int, int]:
    """[start, stop) of rank's contiguous slice; the first global_batch % world ranks get one extra."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    if global_batch < 0:
        raise ValueError("global_batch must be >= 0")
    q, r = divmod(global_batch, world)
    start = rank * q + min(rank, r)
    return start, start + q + (1 if rank < r else 0)


def shard_batch(x: torch.Tensor, rank: int | None = None, world: int | None = None,
                group=None) -> torch.Tensor:
    """This rank's contiguous slice (dim 0) of a batch every rank holds (e.g. z from a shared seed)."""
    if rank is None or world is None:
        rank, world = dist.get_rank(group), dist.get_world_size(group)
    a, b = shard_range(x.shape[0], rank, world)
    return x[a:b]


def broadcast_module(module: torch.nn.Module, src: int = 0, group=None) -> None:
    """Replicate parameters and buffers (running stats, num_batches_tracked) from ``src``."""
    with torch.no_grad():
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, src, group=group)


def enable_sync_bn(group=None, even_world1: bool = False) -> None:
    """Make every train-mode BN of this package use global (all-reduced) batch statistics.
    ``even_world1`` keeps the all-reduce in a one-rank group (tests)."""
    rt.set_sync_bn_group(group if group is not None else dist.group.WORLD, even_world1)


def disable_sync_bn() -> None:
    rt.set_sync_bn_group(None)


def merge_moments(moments: torch.Tensor, group=None) -> torch.Tensor:
    """In-place SUM all-reduce of a (C, 3) float64 tensor of raw moments {n, sum x, sum x^2}.

    Raw moments are additive across disjoint shards, so the merged tensor equals the moments of
    the global batch up to fp64 summation order.  Called by the BN path of ``_runtime`` between
    ``ffc_bn_reduce`` and ``ffc_bn_finalize`` (include/ffc_amd.h)."""
    if moments.dtype != torch.float64 or moments.dim() != 2 or moments.shape[1] != 3:
        raise ValueError(f"moments must be (C, 3) float64, got {tuple(moments.shape)} {moments.dtype}")
    dist.all_reduce(moments, op=dist.ReduceOp.SUM, group=group)
    return moments


def gather_batch(x: torch.Tensor, global_batch: int | None = None, group=None) -> torch.Tensor:
    """all_gather of per-rank slices (possibly ragged, as shard_range makes them) -> global batch."""
    world = dist.get_world_size(group)
    n = torch.tensor([x.shape[0]], device=x.device, dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    if global_batch is not None and sum(sizes) != global_batch:
        raise ValueError(f"shards sum to {sum(sizes)}, expected {global_batch}")
    mx = max(sizes)
    pad = x.new_zeros((mx,) + tuple(x.shape[1:]))
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous(), group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
