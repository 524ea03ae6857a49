"""GPU tests of the launch cut (hpt_render.hip k_trace / k_post, hpt_capi.cpp renderImpl).

A bounce's trace launch whose queues run dry may leave the closest rays its waves are still
tracing unfinished instead of waiting for them (the reference has no such launch boundary: its
per-path loop, path.cpp:135-287, simply goes on).  Their hit records stay pending, k_post moves
the paths to a carry set, the next bounce's launch traces those rays again from their start and
its k_post posts them; a bounce after which no wavefront bounce follows traces the carried rays
in a launch of their own.  A path's arithmetic never depends on which launch traced its ray, so
the film must be bit-identical to the launches that drain every ray (HPT_CUT=0), in the
host-synchronised loop and with bounces launched ahead on a recorded schedule.

HPT_CUT_MIN=0 lets every launch cut (the default cuts only launches with 4 rays per lane): on
these small frames the lanes are dry at their first claim, so nearly every closest ray is carried
once or several times -- the carry sets, the re-carry of carried rays and the flush launch are all
exercised.
"""
import numpy as np
import pytest

import scene_util

pytestmark = pytest.mark.gpu

HAIRCURL_RADII = (0.0025, 0.0025)


def _renders(name, n, radii, monkeypatch, cut, cut_min, tail, ahead="1", times=3, size=(64, 48, 16)):
    monkeypatch.setenv("HPT_CUT", cut)
    monkeypatch.setenv("HPT_CUT_MIN", cut_min)
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)
    monkeypatch.setenv("HPT_BOUNCE_AHEAD", ahead)
    w, h, spp = size
    _, r, _ = scene_util.make(name, n, w, h, spp, device=0, radii=radii)
    out = []
    for _ in range(times):
        film = r.render(0, spp, collect_stats=True)
        out.append((film, r.stats()))
    r.close()
    return out


@pytest.mark.parametrize("name,n,radii", [("furball_marschner", 1500, None), ("straight_kk", 400, None),
                                          ("haircurl_roughplastic", 300, HAIRCURL_RADII)])
@pytest.mark.parametrize("tail", ["0", "2000"])
def test_cut_bit_identical(name, n, radii, tail, monkeypatch):
    (ref, s0), = _renders(name, n, radii, monkeypatch, "0", "4", tail, ahead="0", times=1)
    assert s0.cut_rays == 0 and s0.carry_flushes == 0
    runs = _renders(name, n, radii, monkeypatch, "1", "0", tail)  # HPT_CUT=1 explicitly (the default is off until measured)
    for k, (film, s) in enumerate(runs):
        np.testing.assert_array_equal(film, ref, err_msg=f"render {k}")
        # the same path-bounces are shaded, whichever launch traced their rays (which of them
        # k_tail shades depends on which paths a cut held back: tail_paths may differ)
        assert s.bounces == s0.bounces, k
        assert s.paths == s0.paths
    s1 = runs[0][1]
    assert s1.cut_rays > 0  # the first render (read back bounce by bounce) cut (and flushed when a tail followed)


@pytest.mark.parametrize("after_us", ["3", "40"])
def test_cut_after_partial_drain(after_us, monkeypatch):
    """HPT_CUT_AFTER_US: a wave drains for a while after its dry point and then leaves its
    unfinished closest rays (split by the drain or not) to the next launch."""
    (ref, s0), = _renders("furball_marschner", 1500, None, monkeypatch, "0", "4", "2000", ahead="0", times=1)
    monkeypatch.setenv("HPT_CUT_AFTER_US", after_us)
    runs = _renders("furball_marschner", 1500, None, monkeypatch, "1", "0", "2000")
    for film, s in runs:
        np.testing.assert_array_equal(film, ref)
        assert s.bounces == s0.bounces


def test_cut_host_loop_only(monkeypatch):
    """Cutting with every bounce read back (no schedules): the flush launch ends each wave."""
    (ref, _), = _renders("furball_marschner", 1500, None, monkeypatch, "0", "4", "2000", ahead="0", times=1)
    runs = _renders("furball_marschner", 1500, None, monkeypatch, "1", "0", "2000", ahead="0", times=2)
    for film, s in runs:
        np.testing.assert_array_equal(film, ref)
        assert s.cut_rays > 0 and s.waves_ahead == 0


def test_cut_default_threshold(monkeypatch):
    """At the default threshold a frame whose bounce launches hold several rays per lane cuts
    (a fraction of its rays) and gives the drained frame's film."""
    size = (512, 512, 16)
    (ref, s0), = _renders("furball_marschner", 40000, None, monkeypatch, "0", "4", "131072", ahead="0", times=1,
                          size=size)
    runs = _renders("furball_marschner", 40000, None, monkeypatch, "1", "4", "131072", times=2, size=size)
    for film, s in runs:
        np.testing.assert_array_equal(film, ref)
        assert s.bounces == s0.bounces
    first, second = runs[0][1], runs[1][1]
    assert first.cut_rays > 0 and second.cut_rays > 0
    assert second.waves_ahead == 1 and second.schedule_misses == 0
    # a fraction of the rays: at most one per lane of each launch that cut
    assert first.cut_rays < 0.25 * s0.bounces
