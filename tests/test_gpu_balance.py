"""GPU tests of the work-balanced shard deal (hpt_get_block_costs / hpt_set_block_weights).

Every render counts the path-bounces it shades per owned 32x32 block; their sum is the frame's
path-bounce count (k_shade + k_tail).  With those counts as weights the blocks are re-dealt
longest-first; the shards of the re-dealt frame cover every block once and add up to the
one-shard frame (up to the per-pixel summation order)."""
import numpy as np
import pytest

import scene_util
from mitsuba_amd import distributed, native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tail", ["0", "2000"])
def test_block_costs_and_weighted_deal(tail, monkeypatch):
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)
    W, H, spp, shards = 160, 96, 8, 3
    nb = ((W + 31) // 32) * ((H + 31) // 32)
    _, r, _ = scene_util.make("furball_marschner", 2000, W, H, spp, device=0)
    full = r.render(0, spp, collect_stats=True)
    s = r.stats()
    costs = r.block_costs(nb)
    assert int(costs.sum()) == s.bounces
    assert (costs > 0).sum() >= nb // 2
    assert r.block_costs(nb).sum() == 0  # read and reset
    # the Hilbert-cyclic shards: each counts only its own blocks, the sum is the frame's
    owner = np.array(distributed.block_owner((W + 31) // 32, (H + 31) // 32, shards))
    tot = np.zeros(nb, np.uint64)
    for k in range(shards):
        r.render(0, spp, shard=k, n_shards=shards)
        c = r.block_costs(nb)
        assert (c[owner != k] == 0).all()
        tot += c
    np.testing.assert_array_equal(tot, costs)
    # weighted deal: the same frame
    r.set_block_weights(costs.astype(np.float64))
    owner_w = native.block_deal(W, H, shards, costs.astype(np.float64))
    acc = np.zeros_like(full)
    for k in range(shards):
        acc += r.render(0, spp, shard=k, n_shards=shards)
        c = r.block_costs(nb)
        assert (c[owner_w != k] == 0).all()
        np.testing.assert_array_equal(c[owner_w == k], costs[owner_w == k])
    np.testing.assert_allclose(acc, full, rtol=1e-5, atol=1e-6)
    r.set_block_weights(None)
    again = r.render(0, spp)
    np.testing.assert_array_equal(again, full)
    r.close()
