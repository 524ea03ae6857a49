"""GPU tests of device-side bounce control (hpt_capi.cpp renderImpl).

A wave of paths rendered again (same spp range and shard since the last
prepare) launches its bounces ahead on the schedule recorded the first time:
k_shade / k_trace / k_post read their queue lengths on the device, and the
k_tail launch decides on the device whether it takes its bounce (fewer than
HPT_TAIL_PATHS live paths) or leaves it to k_shade.  The host reads the
counters back once per wave instead of once per bounce.  The schedule only
decides grid sizes and launch order; every path takes the same per-path
steps (path.cpp:119-294), so the film must be bit-identical to the
host-synchronised loop's, whether the schedule fits, is too small (the
overflowing wave is rendered again) or ends a bounce early (the tail
declines and the host goes on bounce by bounce).
"""
import numpy as np
import pytest

import scene_util

pytestmark = pytest.mark.gpu

HAIRCURL_RADII = (0.0025, 0.0025)


def _render_twice(name, n, radii, monkeypatch, ahead, hook, tail, max_wave=0, times=2):
    monkeypatch.setenv("HPT_BOUNCE_AHEAD", ahead)
    monkeypatch.setenv("HPT_SCHEDULE_TEST", hook)
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)
    _, r, _ = scene_util.make(name, n, 64, 48, 16, device=0, radii=radii)
    out = []
    for _ in range(times):
        film = r.render(0, 16, max_wave_paths=max_wave, collect_stats=True)
        out.append((film, r.stats()))
    r.close()
    return out


@pytest.mark.parametrize("name,n,radii", [("furball_marschner", 1500, None), ("straight_kk", 400, None),
                                          ("haircurl_roughplastic", 300, HAIRCURL_RADII)])
@pytest.mark.parametrize("tail", ["0", "2000"])
def test_bounce_ahead_bit_identical(name, n, radii, tail, monkeypatch):
    (ref, s0), _ = _render_twice(name, n, radii, monkeypatch, "0", "0", tail)
    assert s0.waves_ahead == 0 and s0.schedule_misses == 0
    for hook in ("0", "1", "2"):
        (first, s1), (second, s2), (third, s3) = _render_twice(name, n, radii, monkeypatch, "1", hook, tail, times=3)
        np.testing.assert_array_equal(first, ref)
        np.testing.assert_array_equal(second, ref)
        np.testing.assert_array_equal(third, ref)
        # the per-path work is the same whatever the schedule
        for s in (s1, s2):
            assert (s.bounces, s.tail_paths, s.max_bounces) == (s0.bounces, s0.tail_paths, s0.max_bounces), hook
        assert s1.waves_ahead == 0 and s1.schedule_misses == 0  # the first render records the schedule
        if hook == "0":
            assert (s2.waves_ahead, s2.schedule_misses) == (1, 0)
        elif hook == "1":
            # half-size grids: the wave outgrows them (whenever a bounce had more than one
            # block of live paths) and is rendered again from its camera pass
            assert s2.schedule_misses == 1 and s2.waves_ahead == 0
            assert s2.paths == s0.paths and s2.waves == s0.waves
        elif tail != "0":
            # one wavefront bounce short: the tail launched ahead declines its bounce (too many
            # live paths) and the host finishes bounce by bounce, re-recording the schedule as the
            # part launched ahead plus the bounces it read back: the third render runs ahead
            assert s2.schedule_misses == 0 and s2.waves_ahead == 0 and s2.schedule_extensions == 1
            assert (s3.waves_ahead, s3.schedule_misses, s3.schedule_extensions) == (1, 0, 0)
        else:
            # no tail in the schedule: the hook leaves it whole
            assert (s2.waves_ahead, s2.schedule_misses) == (1, 0)


def test_bounce_ahead_several_waves(monkeypatch):
    """A frame of several waves (max_wave_paths): each spp range records its own schedule,
    and the second render launches every wave ahead."""
    (ref, s0), _ = _render_twice("furball_marschner", 1500, None, monkeypatch, "0", "0", "2000", max_wave=1 << 14)
    (first, s1), (second, s2) = _render_twice("furball_marschner", 1500, None, monkeypatch, "1", "0", "2000",
                                              max_wave=1 << 14)
    assert s0.waves > 1
    np.testing.assert_array_equal(first, ref)
    np.testing.assert_array_equal(second, ref)
    assert s2.waves_ahead == s0.waves and s2.schedule_misses == 0
    assert s2.bounces == s0.bounces and s2.tail_paths == s0.tail_paths
