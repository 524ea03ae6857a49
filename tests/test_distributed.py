"""World-size-2 rehearsal of the multi-GPU path on the CPU (gloo backend).

Each rank renders its Hilbert-cyclic shard with the oracle (the GPU renderer's
block ownership, include/hairpt.h hpt_render_params.shard/n_shards, is the
same rule) and mitsuba_amd.distributed.render_frame reduces the films to rank
0, exactly as bench.py does over RCCL.  Rank 0's film must equal the
single-process render up to summation order, every block must be owned by
exactly one rank, and both ranks must have done work.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import scene_util
from mitsuba_amd import distributed, native

W, H, SPP, N = 72, 40, 2, 600  # 3 x 2 blocks of 32x32 (ragged right/bottom edges)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, _, o = scene_util.make("furball_marschner", N, W, H, SPP)

        def render_shard(shard, n_shards, film):
            f, st = o.render(0, SPP, threads=2, shard=shard, n_shards=n_shards, width=W, height=H)
            film += torch.from_numpy(f)
            np.save(os.path.join(out_dir, "shard%d.npy" % rank), f)

        film = torch.zeros((H, W, 4), dtype=torch.float32)
        distributed.render_frame(render_shard, film, rank, world, dist)
        if rank == 0:
            np.save(os.path.join(out_dir, "reduced.npy"), film.numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_block_cyclic_frame(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    reduced = np.load(tmp_path / "reduced.npy")
    s0, s1 = np.load(tmp_path / "shard0.npy"), np.load(tmp_path / "shard1.npy")
    _, _, o = scene_util.make("furball_marschner", N, W, H, SPP)
    full, _ = o.render(0, SPP, threads=2, width=W, height=H)
    np.testing.assert_allclose(reduced, full, rtol=1e-5, atol=1e-6)
    # ownership (distributed.block_owner, Hilbert-cyclic); a shard's film is zero
    # outside its blocks plus the 1-pixel tent border
    nbx = (W + 31) // 32
    owner = distributed.block_owner(nbx, (H + 31) // 32, world)
    for rank, f in ((0, s0), (1, s1)):
        assert f[..., 3].sum() > 0
        for by in range((H + 31) // 32):
            for bx in range(nbx):
                b = by * nbx + bx
                core = f[by * 32 + 1:min(H, by * 32 + 31), bx * 32 + 1:min(W, bx * 32 + 31), 3]
                if owner[b] == rank:
                    assert core.min() > 0
                else:
                    assert core.max() == 0


@pytest.mark.parametrize("nbx,nby", [(16, 16), (32, 32), (38, 32), (2, 2), (1, 3), (5, 1)])
def test_block_order_is_a_balanced_permutation(nbx, nby):
    order = distributed.block_order(nbx, nby)
    assert sorted(order) == list(range(nbx * nby))
    for world in (1, 2, 4, 8):
        owner = distributed.block_owner(nbx, nby, world)
        counts = np.bincount(owner, minlength=world)
        assert counts.max() - counts.min() <= 1
    # a rank's blocks are not whole block columns (the plain b % world deal's flaw)
    if nbx == 16 and nby == 16:
        owner = np.array(distributed.block_owner(nbx, nby, 8)).reshape(nby, nbx)
        for r in range(8):
            assert len(np.unique(np.nonzero(owner == r)[1])) >= 8  # spans at least 8 columns


def _bench_worker(rank, world, port, out_dir):
    """bench.py's own timing helper over gloo: both ranks must report the slower rank's time."""
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []
        dt = bench.timed_steps(lambda: time.sleep(0.02 * (rank + 1)), 3, world, dist, lambda: None, "cpu",
                               after_step=lambda: calls.append(1))
        np.save(os.path.join(out_dir, "dt%d.npy" % rank), np.array([dt, len(calls)]))
    finally:
        dist.destroy_process_group()


def test_bench_timed_steps_takes_max_over_ranks(tmp_path):
    world = 2
    mp.spawn(_bench_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    d0, d1 = np.load(tmp_path / "dt0.npy"), np.load(tmp_path / "dt1.npy")
    assert d0[1] == d1[1] == 3  # exactly K timed steps, each followed by the stats callback
    assert d0[0] == d1[0]       # every rank holds the MAX over ranks
    assert d0[0] >= 3 * 0.04    # ... which is the slower rank's (rank 1 sleeps 40 ms per step)


@pytest.mark.parametrize("w,h,world", [(512, 512, 8), (1024, 1024, 8), (200, 130, 3), (512, 512, 2)])
def test_weighted_deal_matches_mirror(w, h, world):
    """hpt_block_deal (the renderer's work-balanced deal) equals distributed.block_owner_weighted,
    every block is owned once, the ranks' loads are balanced to within one block's weight, and
    without weights it is the Hilbert-cyclic deal."""
    nbx, nby = (w + 31) // 32, (h + 31) // 32
    rng = np.random.default_rng(7)
    weights = rng.gamma(2.0, 1000.0, nbx * nby)
    weights[rng.random(nbx * nby) < 0.2] = 0.0  # empty blocks (no hair)
    got = native.block_deal(w, h, world, weights)
    assert list(got) == distributed.block_owner_weighted(nbx, nby, world, weights)
    loads = np.bincount(got, weights=weights, minlength=world)
    assert loads.max() - loads.min() <= weights.max() + 1e-9
    assert list(native.block_deal(w, h, world)) == distributed.block_owner(nbx, nby, world)


class _FakeCosts:
    """stands in for a Renderer: the blocks this rank owns report their (made-up) work"""

    def __init__(self, costs):
        self.costs, self.weights = costs, None

    def block_costs(self, n):
        return self.costs[:n].copy()

    def set_block_weights(self, w):
        self.weights = np.array(w)


def _balance_worker(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        nbx = nby = 4
        owner = np.array(distributed.block_owner(nbx, nby, world))
        full = np.arange(1, nbx * nby + 1, dtype=np.uint64) * 10
        mine = np.where(owner == rank, full, 0).astype(np.uint64)
        fake = _FakeCosts(mine)
        w = distributed.balance_blocks(fake, nbx * nby, world, dist, "cpu")
        np.save(os.path.join(out_dir, "w%d.npy" % rank), fake.weights)
        assert (w == fake.weights).all()
    finally:
        dist.destroy_process_group()


def test_balance_blocks_sums_costs_over_ranks(tmp_path):
    """bench.py --balance: the ranks' per-block counts (each rank only its own blocks) are summed
    with an all-reduce, and every rank sets the same full weight vector (so the same deal)."""
    world = 2
    mp.spawn(_balance_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    w0, w1 = np.load(tmp_path / "w0.npy"), np.load(tmp_path / "w1.npy")
    np.testing.assert_array_equal(w0, w1)
    np.testing.assert_array_equal(w0, np.arange(1, 17) * 10.0)


def test_block_weights_add_camera_rays():
    """bench.py's deal weighs a block by its path-bounces plus its camera rays (pixels x spp x
    CAMERA_RAY_WEIGHT): a sky block (no bounce) is not free, an edge block has fewer pixels."""
    import numpy as np
    W, H, spp = 80, 40, 16  # 3 x 2 blocks; the last column is 16 pixels wide, the last row 8 high
    costs = np.array([100, 0, 5, 7, 0, 0], np.uint64)
    w = distributed.block_weights(costs, spp, W, H)
    px = np.array([32 * 32, 32 * 32, 16 * 32, 32 * 8, 32 * 8, 16 * 8], np.float64)
    np.testing.assert_allclose(w, costs.astype(np.float64) + distributed.CAMERA_RAY_WEIGHT * spp * px)
    assert w[1] > 0 and w[4] < w[1]


def test_bench_world_size_must_match_gpus():
    """bench.py --gpus N: the launcher's WORLD_SIZE must equal N (a line saying n_gpus N ran N ranks);
    without a launcher N = 1 runs in-process and N > 1 starts the ranks itself (launch_ranks)."""
    import bench
    assert bench.check_world(1, {}) == 1
    assert bench.check_world(4, {"WORLD_SIZE": "4"}) == 4
    with pytest.raises(SystemExit, match="WORLD_SIZE=3"):
        bench.check_world(2, {"WORLD_SIZE": "3"})
    with pytest.raises(SystemExit, match="needs 2 ranks"):
        bench.check_world(2, {})


def test_bench_mismatched_launch_fails_loudly():
    """The whole script exits non-zero, before any device work, when --gpus and WORLD_SIZE disagree."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    res = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--cpu-baseline", "off"], cwd=root, env=env,
                         capture_output=True, text=True, timeout=300)
    assert res.returncode != 0
    assert "WORLD_SIZE=3" in res.stderr
    assert '{"metric"' not in res.stdout
