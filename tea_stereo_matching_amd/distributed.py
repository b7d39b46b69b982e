"""Data-parallel sharding of independent stereo pairs.

Pairs never exchange data, so ranks split the batch with no data-path collective; the
only collective is a gather of the fp32 disparity maps to rank 0 (RCCL over xGMI on
MI355X, `gloo` in the CPU tests) so the caller holds every result.
"""
from __future__ import annotations

import os


def world_info() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(rank: int, pairs_per_rank: int) -> range:
    """Global pair indices owned by `rank` (weak scaling: a fixed batch per rank)."""
    return range(rank * pairs_per_rank, (rank + 1) * pairs_per_rank)


def pair_seed(global_index: int, base: int = 1000) -> int:
    """Synthetic-scene seed of a global pair index (config B pair 0 is seed 1000)."""
    return base + global_index


def gather_to_root(tensor, rank: int, world: int, buffers=None):
    """Gather `tensor` ([B, H, W] disparities) from every rank onto rank 0.

    Returns the list of per-rank tensors on rank 0, None elsewhere.  `buffers` may be
    preallocated on rank 0 (a list of `world` tensors shaped like `tensor`)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return [tensor]
    if rank == 0 and buffers is None:
        buffers = [torch.empty_like(tensor) for _ in range(world)]
    dist.gather(tensor, buffers if rank == 0 else None, dst=0)
    return buffers if rank == 0 else None


def max_over_ranks(value: float, world: int, device=None) -> float:
    """MAX of a float across ranks (the slowest rank defines the step time)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(value: float, world: int, device=None) -> float:
    """MIN of a float across ranks (e.g. a 1/0 verification flag: every rank must pass)."""
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())
