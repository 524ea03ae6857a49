"""Multi-GPU frame rendering: one process per GPU (torch.distributed over RCCL).

The frame's 32x32 blocks (the reference's block size, src/mitsuba/mitsuba.cpp:144)
are dealt block-cyclically: rank r renders every sample of the blocks b with
b % world == r.  Each rank accumulates its samples into its own
full-frame RGBW film -- the tent filter reaches one pixel into neighbouring
blocks, so no border exchange is needed -- and one reduce(sum) to rank 0
combines the films.  Paths never depend on which rank traces them
(Sobol indices depend only on pixel and sample index), so the sharded frame
equals the single-GPU frame up to floating-point summation order.
"""
from __future__ import annotations


def render_frame(render_shard, film, rank: int, world: int, dist=None):
    """render_shard(shard, n_shards, film) accumulates this rank's blocks into
    `film` (a torch tensor; device for RCCL, CPU for gloo); the films are then
    summed on rank 0.  Returns `film` (complete on rank 0 only)."""
    render_shard(rank, world, film)
    if world > 1:
        if dist is None:
            import torch.distributed as dist
        dist.reduce(film, 0)
    return film
