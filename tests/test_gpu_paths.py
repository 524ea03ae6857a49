"""GPU tests of k_paths, the persistent bounce kernel (hpt_render.hip).

A wave of paths with a recorded bounce schedule runs every bounce in one launch: waves of the grid
shade 64 paths at a time into ray chunks, trace rays from any published chunk, and post + shade the
paths whose two rays have finished, with no frame-wide barrier per bounce.  Each path takes the
wavefront loop's per-path steps in the same order (shadePath, the traversal, NEE term then the
emitter term, postPath), and its radiance travels with it, so the film must be bit-identical to
the wavefront loop's (HPT_PATHS=0) for every BSDF, for several hair shapes, with and without a
tail launch in the recorded schedule, over several waves of paths, and when a launch runs out of
chunk capacity (the wave is rendered again by the wavefront loop).
"""
import numpy as np
import pytest

import scene_util

pytestmark = pytest.mark.gpu

HAIRCURL_RADII = (0.0025, 0.0025)


def _renders(name, n, radii, monkeypatch, paths, tail="0", W=64, H=48, spp=16, max_wave=0, times=2, cap=None):
    monkeypatch.setenv("HPT_PATHS", paths)
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)
    if cap is not None:
        monkeypatch.setenv("HPT_PATHS_CAP_TEST", cap)
    else:
        monkeypatch.delenv("HPT_PATHS_CAP_TEST", raising=False)
    _, r, _ = scene_util.make(name, n, W, H, spp, device=0, radii=radii)
    out = []
    for _ in range(times):
        film = r.render(0, spp, max_wave_paths=max_wave, collect_stats=True)
        out.append((film, r.stats()))
    r.close()
    return out


@pytest.mark.parametrize("name,n,radii", [("furball_marschner", 1500, None), ("straight_kk", 400, None),
                                          ("furball_roughplastic", 1500, None), ("straight_dielectric", 400, None),
                                          ("straight_thindielectric", 400, None),
                                          ("haircurl_roughplastic", 300, HAIRCURL_RADII)])
@pytest.mark.parametrize("tail", ["0", "2000"])
def test_paths_kernel_bit_identical(name, n, radii, tail, monkeypatch):
    (ref, s0), _ = _renders(name, n, radii, monkeypatch, "0", tail)
    (first, s1), (second, s2), (third, s3) = _renders(name, n, radii, monkeypatch, "1", tail, times=3)
    np.testing.assert_array_equal(first, ref)  # the first render records the schedule (wavefront)
    np.testing.assert_array_equal(second, ref)
    np.testing.assert_array_equal(third, ref)
    assert s1.paths_launches == 0 and s2.paths_launches == 1 and s3.paths_launches == 1
    assert s2.schedule_misses == 0 and s2.waves_ahead == 1
    # every path-bounce shaded once, whichever kernel shaded it
    assert s2.bounces == s0.bounces and s3.bounces == s0.bounces
    assert s2.ms_paths > 0


def test_paths_kernel_several_waves(monkeypatch):
    """Every wave of a frame with its own schedule runs in its own k_paths launch (a wave whose
    schedule is all k_tail -- fewer live paths than HPT_TAIL_PATHS after the camera pass -- keeps
    its tail launch)"""
    (ref, s0), _ = _renders("furball_marschner", 1500, None, monkeypatch, "0", tail="0", max_wave=1 << 14)
    (first, _), (second, s2) = _renders("furball_marschner", 1500, None, monkeypatch, "1", tail="0",
                                        max_wave=1 << 14)
    assert s0.waves > 1
    np.testing.assert_array_equal(first, ref)
    np.testing.assert_array_equal(second, ref)
    assert s2.paths_launches == s0.waves and s2.bounces == s0.bounces, (
        s2.paths_launches, s2.waves, s2.waves_ahead, s2.schedule_misses, s2.tail_paths, s0.tail_paths, s0.bounces)


def test_paths_kernel_capacity_overflow_renders_again(monkeypatch):
    """A launch whose chunk queues run out aborts every wave; the host renders the wave again with
    the wavefront loop (schedule_misses), and the film is still the reference's."""
    (ref, _), = _renders("furball_marschner", 1500, None, monkeypatch, "0", tail="0", times=1)
    (first, _), (second, s2) = _renders("furball_marschner", 1500, None, monkeypatch, "1", tail="0", cap="64")
    np.testing.assert_array_equal(first, ref)
    np.testing.assert_array_equal(second, ref)
    assert s2.schedule_misses == 1 and s2.paths_launches == 1


def test_paths_kernel_larger_frame(monkeypatch):
    """Hundreds of thousands of paths in flight at once across every XCD: the hand-offs between
    waves (ray chunks, slot states, post chunks) under full load"""
    (ref, s0), = _renders("furball_marschner", 4000, None, monkeypatch, "0", W=256, H=192, spp=64, times=1)
    (first, _), (second, s2) = _renders("furball_marschner", 4000, None, monkeypatch, "1", W=256, H=192, spp=64)
    np.testing.assert_array_equal(first, ref)
    np.testing.assert_array_equal(second, ref)
    assert s2.paths_launches == 1 and s2.bounces == s0.bounces
