"""Multi-GPU frame rendering: one process per GPU (torch.distributed over RCCL).

The frame's 32x32 blocks (the reference's block size, src/mitsuba/mitsuba.cpp:144)
are dealt cyclically along a Hilbert curve over the block grid: rank r renders
every sample of the blocks at positions r, r + world, r + 2 world, ... of that
curve (block_owner below; hpt_capi.cpp blockOrder is the renderer's own copy).
N consecutive blocks of the curve form a compact patch, so every rank gets one
block of every patch and the hair's uneven screen coverage is spread evenly
(SURVEY.md 8e's plain b % world deal hands whole block columns to a rank
whenever world divides the number of block columns: 0.73 strong-scaling
efficiency at 8 ranks on the headline frame).  Each rank accumulates its samples into its own
full-frame RGBW film -- the tent filter reaches one pixel into neighbouring
blocks, so no border exchange is needed -- and one reduce(sum) to rank 0
combines the films.  Paths never depend on which rank traces them
(Sobol indices depend only on pixel and sample index), so the sharded frame
equals the single-GPU frame up to floating-point summation order.
"""
from __future__ import annotations


def block_order(nbx: int, nby: int) -> list[int]:
    """Image blocks (by * nbx + bx) in Hilbert-curve order over the nbx x nby grid."""
    n = 1
    while n < max(nbx, nby):
        n <<= 1
    order = []
    for d in range(n * n):
        x = y = 0
        t = d
        sq = 1
        while sq < n:
            rx = 1 & (t // 2)
            ry = 1 & (t ^ rx)
            if ry == 0:
                if rx == 1:
                    x, y = sq - 1 - x, sq - 1 - y
                x, y = y, x
            x += sq * rx
            y += sq * ry
            t //= 4
            sq <<= 1
        if x < nbx and y < nby:
            order.append(y * nbx + x)
    return order


def block_owner(nbx: int, nby: int, world: int) -> list[int]:
    """owner[b] = rank that renders 32x32 block b (hpt_render_params.shard / n_shards)."""
    owner = [0] * (nbx * nby)
    for k, b in enumerate(block_order(nbx, nby)):
        owner[b] = k % world
    return owner


def block_owner_weighted(nbx: int, nby: int, world: int, weights) -> list[int]:
    """The work-balanced deal (hpt_capi.cpp dealBlocks, hpt_set_block_weights): blocks by
    descending weight (ties in Hilbert order), each to the rank with the least weight so far
    (ties to the lowest rank).  weights[b] is block b's measured work."""
    order = block_order(nbx, nby)
    pos = sorted(range(len(order)), key=lambda i: -float(weights[order[i]]))  # stable: Hilbert ties
    load = [0.0] * world
    owner = [0] * (nbx * nby)
    for i in pos:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[order[i]] = r
        load[r] += float(weights[order[i]])
    return owner


# A block's camera pass in path-bounce units: the headline frame's camera pass (quadrant packets,
# 23.4 ms for 67 M camera rays) against its bounces (trace + shade + post + tail, 110.8 ms for
# 113 M path-bounces): 0.36 of a path-bounce per camera ray (0.44 before the quadrant packets).  Sky blocks shade no bounce, but each
# of their pixels still costs its camera rays.
CAMERA_RAY_WEIGHT = 0.36


def block_weights(costs, spp: int, width: int, height: int, block: int = 32):
    """Per-block work for the deal: the path-bounces a block shaded (hpt_get_block_costs)
    plus its camera rays (its pixels x spp) weighted by CAMERA_RAY_WEIGHT."""
    import numpy as np
    nbx, nby = (width + block - 1) // block, (height + block - 1) // block
    bx, by = np.meshgrid(np.arange(nbx), np.arange(nby))
    pixels = (np.minimum(block, width - bx * block) * np.minimum(block, height - by * block)).ravel()
    return np.asarray(costs, np.float64) + CAMERA_RAY_WEIGHT * spp * pixels.astype(np.float64)


def balance_blocks(renderer, n_blocks: int, world: int, dist=None, device=None, spp=None, width=None, height=None,
                   frames: int = 1):
    """After a frame: every rank reads the path-bounces its blocks shaded
    (hpt_get_block_costs), the counts are summed over ranks, and every rank sets the same
    weights (hpt_set_block_weights; with spp / width / height the camera rays are added, see
    block_weights), so the next frames use the same work-balanced deal.  The device counts
    add up over every render since the last read: `frames` is how many frames of spp samples
    they cover (they are divided by it, so the per-frame camera-ray term of block_weights
    keeps its weight).  Returns the weights."""
    import numpy as np
    import torch
    if frames < 1:
        raise ValueError("balance_blocks: the costs must cover at least one frame")
    costs = renderer.block_costs(n_blocks).astype(np.float64) / float(frames)
    if world > 1:
        if dist is None:
            import torch.distributed as dist
        t = torch.tensor(costs, dtype=torch.float64, device=device)
        dist.all_reduce(t)
        costs = t.cpu().numpy()
    if spp is not None:
        costs = block_weights(costs, spp, width, height)
    renderer.set_block_weights(costs)
    return costs


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
