"""GPU tests of the resumable cut (hpt_kernels.h HPT_C_CARRY_*, BounceIO in hpt_render.hip).

A bounce's trace launch whose queue runs dry saves the traversal state of every ray still
running (ray, interval, best hit, node, ring stack, round count) instead of draining it; the
next launch resumes it first, and the bounce's k_post holds the ray's path back until both of
its rays are done.  Each ray therefore tests the same segments in the same order with the
same intervals, and each path adds its NEE term before its emitter term (path.cpp:119-294):
the film must be bit-identical to the drained render, with the rays cut and resumed any
number of times (HPT_CUT_MIN low: small launches cut at once, resumed rays are cut again;
the cut stops at the bounce where Russian roulette starts),
in the read-back loop and with the bounces launched ahead, with and without k_tail, for one
and several hair shapes, and over several waves of paths.
"""
import numpy as np
import pytest

import scene_util

pytestmark = pytest.mark.gpu

HAIRCURL_RADII = (0.0025, 0.0025)


def _render(name, n, radii, monkeypatch, cut_min, tail, ahead, times=1, w=64, h=48, spp=16, max_wave=0):
    monkeypatch.setenv("HPT_CUT_MIN", str(cut_min))
    monkeypatch.setenv("HPT_TAIL_PATHS", tail)
    monkeypatch.setenv("HPT_CUT_TAIL", tail)  # (the shipped one, 2^19, would take these small frames whole)
    monkeypatch.setenv("HPT_BOUNCE_AHEAD", ahead)
    _, r, _ = scene_util.make(name, n, w, h, spp, device=0, radii=radii)
    out = []
    for _ in range(times):
        film = r.render(0, spp, max_wave_paths=max_wave, collect_stats=True)
        out.append((film, r.stats()))
    r.close()
    return out


@pytest.mark.parametrize("name,n,radii", [("furball_marschner", 1500, None), ("straight_kk", 400, None),
                                          ("haircurl_roughplastic", 300, HAIRCURL_RADII)])
@pytest.mark.parametrize("tail", ["0", "2000"])
def test_cut_bit_identical(name, n, radii, tail, monkeypatch):
    [(ref, s0)] = _render(name, n, radii, monkeypatch, 0, tail, "0")
    assert s0.cut_rays == 0
    # read back per bounce, then launched ahead on the recorded schedule (twice)
    (f1, s1), (f2, s2), (f3, s3) = _render(name, n, radii, monkeypatch, 1000, tail, "1", times=3)
    assert s1.cut_rays > 0, "the forced cut must cut"
    for f in (f1, f2, f3):
        np.testing.assert_array_equal(f, ref)
    for s in (s1, s2, s3):
        # the same path-bounces whatever the cut held back; k_tail takes the same paths
        assert (s.bounces, s.paths) == (s0.bounces, s0.paths)


def test_cut_several_waves(monkeypatch):
    # (waves of 2^14 paths: a few thousand rays per launch, so the threshold is lowered further)
    [(ref, s0)] = _render("furball_marschner", 1500, None, monkeypatch, 0, "0", "0", max_wave=1 << 14)
    (f1, s1), (f2, s2) = _render("furball_marschner", 1500, None, monkeypatch, 100, "0", "1", times=2,
                                 max_wave=1 << 14)
    assert s0.waves > 1 and s1.cut_rays > 0
    np.testing.assert_array_equal(f1, ref)
    np.testing.assert_array_equal(f2, ref)
    assert s1.bounces == s0.bounces and s2.bounces == s0.bounces


def test_cut_default_threshold_large_frame(monkeypatch):
    """at 2^18 closest rays and the 2^17 tail a 256x256 @ 64 frame of 4 M paths cuts its first
    bounces' launches on its own; the film equals the drained one bit for bit"""
    [(ref, s0)] = _render("furball_marschner", 8000, None, monkeypatch, 0, str(1 << 17), "1", w=256, h=256, spp=64)
    (f1, s1), (f2, s2) = _render("furball_marschner", 8000, None, monkeypatch, 1 << 18, str(1 << 17), "1", times=2,
                                 w=256, h=256, spp=64)
    assert s1.cut_rays > 0 and s2.cut_rays > 0
    np.testing.assert_array_equal(f1, ref)
    np.testing.assert_array_equal(f2, ref)
    # the same path-bounces; k_tail may start a bounce later (it takes no held-back work)
    assert s1.bounces == s0.bounces and s2.bounces == s0.bounces
