"""GPU tests of k_trace's claim-order buckets (HPT_CLAIM_BUCKETS, hpt_kernels.h HPT_BUCKETS).

k_shade appends each bounce ray to one of four buckets by the length of its interval inside
the scene box, and k_trace's cursor shards claim the longest bucket first, so that the rays
still running when the launch's queue runs dry are short ones.  Only the order in which rays
are claimed changes: every ray is traced by the same traversal with the same interval, a
path's shadow ray and continuation ray write different words, so the film must be
bit-identical to the queue-order launch's, for one wave, several waves and sharded frames.
"""
import numpy as np
import pytest

import scene_util

pytestmark = pytest.mark.gpu


def _render(name, n, monkeypatch, buckets, w=64, h=48, spp=16, tail="0", **kw):
    monkeypatch.setenv("HPT_CLAIM_BUCKETS", buckets)
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)  # "0": every bounce a wavefront trace launch
    _, r, _ = scene_util.make(name, n, w, h, spp, device=0)
    film = r.render(0, spp, collect_stats=True, **kw)
    s = r.stats()
    r.close()
    return film, s


@pytest.mark.parametrize("name,n", [("furball_marschner", 1500), ("straight_kk", 400)])
@pytest.mark.parametrize("tail", ["0", "2000"])
def test_claim_buckets_bit_identical(name, n, tail, monkeypatch):
    ref, s0 = _render(name, n, monkeypatch, "0", tail=tail)
    film, s1 = _render(name, n, monkeypatch, "1", tail=tail)
    np.testing.assert_array_equal(film, ref)
    assert (s1.bounces, s1.tail_paths, s1.max_bounces) == (s0.bounces, s0.tail_paths, s0.max_bounces)


def test_claim_buckets_waves_and_shards(monkeypatch):
    ref, _ = _render("furball_marschner", 3000, monkeypatch, "0", 96, 64, 32, max_wave_paths=1 << 15)
    film, s = _render("furball_marschner", 3000, monkeypatch, "1", 96, 64, 32, max_wave_paths=1 << 15)
    assert s.waves > 1
    np.testing.assert_array_equal(film, ref)
    for shard in range(3):
        a, _ = _render("furball_marschner", 3000, monkeypatch, "0", 96, 64, 32, shard=shard, n_shards=3)
        b, _ = _render("furball_marschner", 3000, monkeypatch, "1", 96, 64, 32, shard=shard, n_shards=3)
        np.testing.assert_array_equal(a, b)
