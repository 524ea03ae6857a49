"""GPU parity on the BASELINE configs that run at 1024^2 (C4 curly, C5 furball-1M).

BASELINE.json configs[3] (models/curly-hair, Marschner, 1024x1024 @ 256 spp,
helical hair of ~2.7e6 segments, models/curly-hair/scene.xml:12,31-38) and
configs[4] (furball scaled to ~1e6 segments, 1024x1024 @ 1024 spp, maxDepth
64).  Both select the Sobol pixel resolution 1024 (m = 10, sobol.cpp:147-158)
and build the deepest kd-trees of the configs.

  - reduced size, same generator and radius: GPU film vs the oracle at the
    reference-flags noise floor (scene_util.reference_flags_floor);
  - full size: the frame is deterministic and invariant under shard and spp
    splits; at full resolution (the m = 10 look-up) a quarter of the blocks at
    64 spp matches the oracle at the floor;
  - the traversal bounds (2^18 leaf rounds, 1024 kd-restarts per ray) fail a
    render loudly (HPT_ETRAVERSAL): every render here passing proves they
    never fired, and the counted frame reports how far below them the longest
    ray stayed.
"""
import numpy as np
import pytest

import scene_util
from mitsuba_amd import native

pytestmark = pytest.mark.gpu


def _parity(name, n, r, o, w, h, spp, max_depth=None, factor=2.0, shard=0, n_shards=1, workdir=None):
    film = r.render(0, spp, shard=shard, n_shards=n_shards, collect_stats=2)
    s = r.stats()
    ofilm, ostats = o.render(0, spp, threads=16, shard=shard, n_shards=n_shards, width=w, height=h)
    np.testing.assert_allclose(film[..., 3], ofilm[..., 3], rtol=1e-5)
    mask = film[..., 3] > 0  # the shard's pixels
    a, b = native.develop(film)[mask], native.develop(ofilm)[mask]
    m = scene_util.l2_metrics(b, a)
    same = np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7, axis=-1)
    floor, floor_same = scene_util.reference_flags_floor(name, n, r, w, h, spp, max_depth=max_depth, shard=shard,
                                                         n_shards=n_shards, workdir=workdir)
    print(name, n, (w, h, spp), "gpu vs oracle", m, "identical %.4f" % same.mean(), "| floor", floor,
          "identical %.4f" % floor_same, "| longest ray: %d leaf rounds, %d restarts, %d rays restarted"
          % (s.max_leaf_rounds, s.max_restarts, s.restarted_rays))
    scene_util.assert_at_floor(m, floor, same.mean(), floor_same, factor=factor)
    assert s.max_leaf_rounds < (1 << 18) and s.max_restarts < 1024
    return s


def test_sobol_m10_bit_exact():
    """hpt_sobol_batch at the 1024^2 configs' look-up resolution (m = 10) and its
    neighbours, over every frame bit a 1024-spp render uses, vs the oracle."""
    _, r, o = scene_util.make("furball_marschner", 300, 1024, 1024, 4, device=0)
    rng = np.random.default_rng(10)
    n = 200000
    for m in (9, 10, 11):
        frame = rng.integers(0, 1024, n).astype(np.uint32)
        px = rng.integers(0, 1 << m, n).astype(np.uint32)
        py = rng.integers(0, 1 << m, n).astype(np.uint32)
        dim = rng.integers(0, 1024, n).astype(np.uint32)
        frame[:4], px[:4], py[:4], dim[:4] = [0, 1023, 512, 1], [0, (1 << m) - 1, 3, 0], [0, (1 << m) - 1, 7, 0], \
            [0, 1023, 2, 1]
        gi, gv = r.sobol(m, frame, px, py, dim)
        oi = o.sobol_lookup(m, frame, px, py)
        np.testing.assert_array_equal(gi, oi)
        np.testing.assert_array_equal(gv, o.sobol_sample(oi, dim))


def test_curly_reduced_matches_oracle():
    """C4 geometry generator and radius at 2,000 strands (5.4e5 segments), 128x96 @ 8 spp."""
    _, r, o = scene_util.make("curly_marschner", 2000, 128, 96, 8, device=0)
    assert r.info().segments > 500000
    _parity("curly_marschner", 2000, r, o, 128, 96, 8)


def test_furball_1m_reduced_matches_oracle():
    """C5 geometry (125,000 strands, ~1e6 segments) and maxDepth 64 at 128x96 @ 8 spp."""
    _, r, o = scene_util.make("furball_1m", 125000, 128, 96, 8, max_depth=64, device=0)
    si = r.info()
    assert si.segments > 900000 and si.max_depth == 64
    _parity("furball_1m", 125000, r, o, 128, 96, 8, max_depth=64)


def test_folded_strands_match_oracle_and_keep_the_pretest(monkeypatch):
    """A furball with an exact hairpin, a one-ulp near-hairpin and a 179.9 degree fold near the
    camera (scene_util.fold_workdir; hair.cpp:485-548,551-596: the miter planes of a fold are
    almost parallel to the axis, or NaN for the exact hairpin): the film matches the oracle at the
    reference-flags floor, and -- the near-hairpin's records flagged to pass instead of widening
    the scene's pre-test radius -- the fp64 exact tests per traced ray stay within 5 % of the
    fold-free twin's (one global bound would have tested every record of the scene at the
    near-hairpin's ~150 radii).  Every bounce goes
    through k_trace (HPT_TAIL_PATHS=0: no k_tail), whose counters the ratio reads."""
    monkeypatch.setenv("HPT_TAIL_PATHS", "0")
    n, w, h, spp = 3000, 128, 96, 8
    per_ray = {}
    for folded in (False, True):
        d = scene_util.fold_workdir(n, folded)
        _, r, o = scene_util.make("furball_marschner", n, w, h, spp, device=0, workdir=d)
        rec, radius, n_pass = r.pretest_records()
        s = _parity("furball_marschner", n, r, o, w, h, spp, workdir=d)
        per_ray[folded] = s.prim_exact / (s.closest_rays + s.shadow_rays)
        print("folded" if folded else "fold-free", "pre-test radius / r %.5f" % (radius / 0.00216667),
              "records flagged to pass %d of %d" % (n_pass, len(rec)), "exact tests per ray %.4f" % per_ray[folded])
        if folded:
            assert n_pass > 0 and radius < 1.05 * 0.00216667
    assert per_ray[True] <= 1.05 * per_ray[False], per_ray


def _full_size(name, n, w, h, spp, max_depth, parity_spp=64):
    _, r, o = scene_util.make(name, n, w, h, spp, max_depth=max_depth, device=0)
    si = r.info()
    print(name, "segments", si.segments, "kd nodes", si.kd_nodes, "depth", si.kd_depth,
          "build %.2f s" % si.kd_build_seconds)
    a = r.render(0, spp)
    np.testing.assert_array_equal(a, r.render(0, spp))
    s = r.render(0, spp, shard=0, n_shards=3)
    s = r.render(0, spp, shard=1, n_shards=3, film=s)
    s = r.render(0, spp, shard=2, n_shards=3, film=s)
    np.testing.assert_allclose(s, a, rtol=1e-5, atol=1e-5)
    c = r.render(0, spp // 3)
    c = r.render(spp // 3, spp, film=c)
    np.testing.assert_allclose(c, a, rtol=1e-5, atol=1e-5)
    img = native.develop(a)
    assert np.all(np.isfinite(img)) and img.mean() > 0
    # full resolution (the m = 10 look-up) vs the oracle: one Hilbert-dealt quarter of the
    # 32x32 blocks (the 4-GPU shard 0) at 64 spp, where a flipped discrete event (a path
    # that reaches the sun on one side only) is averaged like the headline's samples
    _parity(name, n, r, o, w, h, parity_spp, max_depth=max_depth, factor=3.0, shard=0, n_shards=4)
    return si


def test_straight_kk_full_size():
    """C2 at full size (BASELINE.json configs[1]): models/straight-hair with Kajiya-Kay,
    10,000 strands, 256x256 @ 64 spp: deterministic, shard- and spp-split invariant, and
    the whole frame at 64 spp against the oracle at the reference-flags floor."""
    _, r, o = scene_util.make("straight_kk", 10000, 256, 256, 64, device=0)
    si = r.info()
    print("straight_kk segments", si.segments, "kd nodes", si.kd_nodes)
    a = r.render(0, 64)
    np.testing.assert_array_equal(a, r.render(0, 64))
    s = r.render(0, 64, shard=0, n_shards=3)
    s = r.render(0, 64, shard=1, n_shards=3, film=s)
    s = r.render(0, 64, shard=2, n_shards=3, film=s)
    np.testing.assert_allclose(s, a, rtol=1e-5, atol=1e-5)
    c = r.render(0, 20)
    c = r.render(20, 64, film=c)
    np.testing.assert_allclose(c, a, rtol=1e-5, atol=1e-5)
    assert np.all(np.isfinite(native.develop(a)))
    _parity("straight_kk", 10000, r, o, 256, 256, 64, factor=2.0)


def test_traversal_bound_fails_loudly_and_recovers():
    """A ray that exceeds the traversal bound (here lowered to 2 leaf rounds through the
    test hook) sets the fault word: the render fails with HPT_ETRAVERSAL (-5) instead of
    returning a film with wrong hits, and the next call, with the bound restored, clears
    the word and succeeds with the reference film."""
    _, r, _ = scene_util.make("furball_marschner", 1500, 32, 24, 2, device=0)
    ref = r.render(0, 2)
    r.set_traversal_bounds(2, 1024)
    with pytest.raises(native.HairPTError) as ei:
        r.render(0, 2)
    assert ei.value.code == -5 and "leaf rounds" in str(ei.value)
    r.set_traversal_bounds()
    np.testing.assert_array_equal(r.render(0, 2), ref)
    # the kd-restart bound the same way: a restart is needed only after a ring-stack
    # overflow, so a zero-restart bound fires on the deep rays of a full-size tree
    _, r2, _ = scene_util.make("furball_marschner", 40000, 64, 64, 4, device=0)
    r2.set_traversal_bounds(1 << 18, 0)
    film = None
    try:
        film = r2.render(0, 4, collect_stats=2)
    except native.HairPTError as e:
        assert e.code == -5 and "restart" in str(e)
    if film is not None:  # no ray overflowed the stack in this frame
        assert r2.stats().restarted_rays == 0
    r2.set_traversal_bounds()
    assert np.isfinite(r2.render(0, 4)).all()


def test_packet_overflow_launch_is_bit_identical():
    """Camera packets whose stack overflows hand their rays to k_trace_overflow (one lane per
    ray, k_trace's traversal) instead of tracing them inside the packet kernel.  With the
    packet stack limited to 1 and 3 entries (test hook) most packets overflow; the film must
    equal the default render bit for bit, and the counted frame must see the overflows."""
    _, r, _ = scene_util.make("furball_marschner", 40000, 64, 48, 8, device=0)
    ref = r.render(0, 8)
    for entries in (1, 3):
        r.set_packet_stack(entries)
        film = r.render(0, 8, collect_stats=2)
        assert r.stats().packet_fallbacks > 0
        np.testing.assert_array_equal(film, ref)
    r.set_packet_stack(0)
    np.testing.assert_array_equal(r.render(0, 8, collect_stats=2), ref)
    assert r.stats().packet_fallbacks == 0


def test_curly_full_size():
    """C4 at full size: 10,000 helical strands (~2.7e6 segments), 1024x1024 @ 256 spp."""
    si = _full_size("curly_marschner", 10000, 1024, 1024, 256, 65)
    assert si.segments > 2600000


def test_furball_1m_full_size():
    """C5 at full size: 125,000 strands, 1024x1024 @ 1024 spp, maxDepth 64."""
    si = _full_size("furball_1m", 125000, 1024, 1024, 1024, 64)
    assert si.segments > 900000


def test_unlimited_depth_delta_only():
    """maxDepth = -1 (the reference's default, 'unlimited') with a delta-only BSDF
    of unit weights (thindielectric, reflectance = transmittance = 1: no NEE, 3
    Sobol dimensions per bounce, throughput stays 1) through the dense furball:
    paths cross fiber after fiber until Russian roulette (q = 0.95) ends them,
    long past the old 8-bit depth field."""
    _, r, o = scene_util.make("furball_thin_white", 40000, 48, 40, 64, max_depth=-1, device=0)
    assert r.info().max_depth == -1
    film = r.render(0, 64, collect_stats=True)
    st = r.stats()
    ofilm, _ = o.render(0, 64, threads=16, width=48, height=40)
    m = scene_util.l2_metrics(native.develop(ofilm), native.develop(film))
    print("unlimited depth: path-bounces", st.bounces, "max bounce launches", st.max_bounces, m)
    assert m["rmse"] < 1e-3, m


def test_zero_segment_hair_renders_environment(tmp_path):
    """A hair file of single-vertex strands loads with zero segments (hair.cpp:663-716):
    the kd-tree is one empty leaf with an inverted AABB, every ray misses, nothing
    faults, and the film is the environment alone."""
    path = str(tmp_path / "singles.txt")
    open(path, "wb").write(b"1 2 3\n\n4 5 6\n\n7 8 9\n")
    r = native.Renderer(device=0)
    r.set_hair_file(path, 0.01, 1.0)
    r.set_camera(np.eye(4, dtype=np.float32), 40, 16, 16)
    r.set_kajiyakay((0.2, 0.2, 0.2))
    r.set_sunsky((0, 1, 0))
    r.prepare()
    assert r.info().segments == 0
    film = r.render(0, 4)
    assert np.all(np.isfinite(film)) and np.all(film[..., 3] > 0)
    assert film[..., :3].max() > 0
    st = r.stats()
    assert st.prims == 0
