"""GPU parity: HIP kernels (through the C ABI) vs the oracle on identical inputs.

Tolerances:
  - Sobol index/values, kd-tree hits (segment id, t, hit point): bit-exact.
  - BSDF / envmap values: float32 transcendental functions differ between
    ROCm's ocml and glibc by <= ~2 ulp, so values are compared with
    rtol 2e-5 and discrete outcomes (sampled lobe/type) must agree for
    > 99.9 % of samples.
  - Rendered film: per-pixel L2 on linear HDR RGB, RMSE < 1e-3 relative to
    mean luminance (north_star "per-pixel L2 error < 1e-3").
"""
import os

import numpy as np
import pytest

import oracle_lib
import scene_util
from mitsuba_amd import distributed, native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def furball():
    xml, r, o = scene_util.make("furball_marschner", 3000, 48, 40, 8, device=0)
    return xml, r, o


@pytest.fixture(scope="module")
def straight():
    xml, r, o = scene_util.make("straight_kk", 1500, 48, 40, 8, device=0)
    return xml, r, o


def test_sobol_bit_exact(furball):
    _, r, o = furball
    rng = np.random.default_rng(1)
    n = 20000
    m = 6
    frame = rng.integers(0, 1000, n).astype(np.uint32)
    px = rng.integers(0, 64, n).astype(np.uint32)
    py = rng.integers(0, 64, n).astype(np.uint32)
    dim = rng.integers(0, 400, n).astype(np.uint32)
    gi, gv = r.sobol(m, frame, px, py, dim)
    oi = o.sobol_lookup(m, frame, px, py)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gv, o.sobol_sample(oi, dim))


def _rays(o, n, seed, width=48, height=40, centre=(0.0, 12.3, 0.0), spread=2.0):
    rng = np.random.default_rng(seed)
    pos = np.stack([rng.uniform(0, width, n // 2), rng.uniform(0, height, n // 2)], 1)
    co, cd, cmin, cmax = o.camera_rays(pos)
    centre = np.array(centre)
    a = centre + rng.normal(0, spread, (n // 2, 3))
    b = centre + rng.normal(0, spread, (n // 2, 3))
    d = (b - a) / np.linalg.norm(b - a, axis=1, keepdims=True)
    orig = np.concatenate([co, a]).astype(np.float32)
    dirs = np.concatenate([cd, d]).astype(np.float32)
    mint = np.concatenate([cmin, np.full(n // 2, 1e-4, np.float32)])
    maxt = np.concatenate([cmax, np.full(n // 2, np.inf, np.float32)])
    return orig, dirs, mint, maxt


def _grazing_rays(r, n, seed, radius, vrange=None):
    """Rays whose line passes the axis of a random segment at radius * (1 +- 1e-4),
    from origins 0.05..40 units away: the worst case for the fp32 pre-test
    (HptSegF in hpt_device.h), which must never reject a segment the exact
    fp64 test accepts."""
    rng = np.random.default_rng(seed)
    xyz, st = r.hair()
    segs = np.nonzero(st[1:len(xyz)] == 0)[0]
    if vrange is not None:  # segments of one hair shape
        segs = segs[(segs >= vrange[0]) & (segs < vrange[1])]
    s = rng.choice(segs, n)
    v1, v2 = xyz[s].astype(np.float64), xyz[s + 1].astype(np.float64)
    axis = (v2 - v1) / np.linalg.norm(v2 - v1, axis=1, keepdims=True)
    q = rng.normal(size=(n, 3))
    u = q - axis * np.sum(q * axis, 1, keepdims=True)
    u /= np.linalg.norm(u, axis=1, keepdims=True)
    w = np.cross(axis, u)
    # direction perpendicular to u: mixes the axis and the third frame vector
    ang = rng.uniform(0.05, np.pi - 0.05, n)[:, None]
    d = np.cos(ang) * axis + np.sin(ang) * w
    f = rng.uniform(0, 1, n)[:, None]
    dist = radius * (1 + rng.uniform(-1e-4, 1e-4, n))[:, None]
    pt = v1 + f * (v2 - v1) + u * dist
    L = np.exp(rng.uniform(np.log(0.05), np.log(40.0), n))[:, None]
    orig = (pt - d * L).astype(np.float32)
    return orig, d.astype(np.float32), np.full(n, 1e-4, np.float32), np.full(n, np.inf, np.float32)


@pytest.mark.parametrize("fixture", ["furball", "straight", "haircurl"])
@pytest.mark.parametrize("kind", ["mixed", "grazing"])
def test_trace_bit_exact(fixture, kind, request):
    _, r, o = request.getfixturevalue(fixture)
    if kind == "mixed":
        orig, dirs, mint, maxt = (_rays(o, 40000, 3, centre=(0.0, 6.0, 0.0), spread=3.0) if fixture == "haircurl"
                                  else _rays(o, 40000, 3))
    elif fixture == "haircurl":
        # grazing rays at each shape's own radius: the shapes' vertex ranges in the merged set
        counts = []
        for path, rad, _ in scene_util.oracle_shapes("haircurl_roughplastic", 300, radii=HAIRCURL_RADII):
            oo = oracle_lib.Oracle()
            oo.check(oo.lib.orc_load_hair(oo.s, path.encode(), rad, 1.0, None))
            counts.append(int(oo.lib.orc_hair_vertex_count(oo.s)))
        first = np.concatenate([[0], np.cumsum(counts)])
        parts = [_grazing_rays(r, 10000, 5 + k, rad, vrange=(first[k], first[k + 1]))
                 for k, rad in enumerate(HAIRCURL_RADII)]
        orig, dirs, mint, maxt = (np.concatenate([p[i] for p in parts]) for i in range(4))
    else:
        name = {"furball": "furball_marschner", "straight": "straight_kk"}[fixture]
        orig, dirs, mint, maxt = _grazing_rays(r, 40000, 5, float(scene_util.scenes.CONFIGS[name]["radius"]))
    gt, giv, gp = r.trace(orig, dirs, mint, maxt)
    ot, oiv, op = o.trace(orig, dirs, mint, maxt)
    assert (oiv >= 0).sum() > 1000
    np.testing.assert_array_equal(giv, oiv)
    np.testing.assert_array_equal(gt, ot)
    np.testing.assert_array_equal(gp, op)
    sm = np.minimum(maxt, 3.0).astype(np.float32)
    osh = o.trace(orig, dirs, mint, sm, shadow=True)
    np.testing.assert_array_equal(r.trace(orig, dirs, mint, sm, shadow=True), osh)
    # packet traversal on incoherent rays: packets split on every order disagreement and
    # overflow their stack (lanes then finish alone) -- the hits must not change
    pt_, piv, pp = r.trace(orig, dirs, mint, maxt, packet=True)
    np.testing.assert_array_equal(piv, oiv)
    np.testing.assert_array_equal(pt_, ot)
    np.testing.assert_array_equal(pp, op)
    # kd-restart path: a 2-entry stack overflows constantly and must give the same answers
    tt, tiv, tp = r.trace(orig, dirs, mint, maxt, tiny_stack=True)
    np.testing.assert_array_equal(tiv, oiv)
    np.testing.assert_array_equal(tt, ot)
    np.testing.assert_array_equal(r.trace(orig, dirs, mint, sm, shadow=True, tiny_stack=True), osh)
    # drain splitting (every batch ends in a drain: idle lanes take over the farthest pending
    # subtrees of running rays) gives the answers of the unsplit traversal
    ut, uiv, up = r.trace(orig, dirs, mint, maxt, split=False)
    np.testing.assert_array_equal(uiv, oiv)
    np.testing.assert_array_equal(ut, ot)
    np.testing.assert_array_equal(up, op)
    np.testing.assert_array_equal(r.trace(orig, dirs, mint, sm, shadow=True, split=False), osh)


@pytest.mark.parametrize("n", [1, 7, 63, 65, 300])
def test_trace_small_batches_split(furball, n):
    """Drain splitting at its most aggressive: a batch of n rays leaves most lanes of
    every wave idle from the start, so running rays are split again and again (stack
    steals and, once a ray's stack is empty, interval halves from the root) -- the
    closest hits, the far roots and the any-hit answers must still be the oracle's and
    the unsplit traversal's (tiny-stack rays split too: lost entries go to the helper)."""
    _, r, o = furball
    # camera rays and random chords (_rays: n // 2 of each), then n grazing rays
    a = _rays(o, n, 100 + n)
    g = _grazing_rays(r, n, 200 + n, float(scene_util.scenes.CONFIGS["furball_marschner"]["radius"]))
    orig, dirs, mint, maxt = (np.concatenate([x, y]).astype(np.float32) for x, y in zip(a, g))
    ot, oiv, op = o.trace(orig, dirs, mint, maxt)
    sm = np.minimum(maxt, 3.0).astype(np.float32)
    osh = o.trace(orig, dirs, mint, sm, shadow=True)
    for kw in ({}, {"split": False}, {"tiny_stack": True}):
        gt, giv, gp = r.trace(orig, dirs, mint, maxt, **kw)
        np.testing.assert_array_equal(giv, oiv, err_msg=str(kw))
        np.testing.assert_array_equal(gt, ot, err_msg=str(kw))
        np.testing.assert_array_equal(gp, op, err_msg=str(kw))
        np.testing.assert_array_equal(r.trace(orig, dirs, mint, sm, shadow=True, **kw), osh, err_msg=str(kw))


HAIRCURL_RADII = [0.02, 0.035, 0.05, 0.028]


def _packet_rays(r, n_groups, seed, cone):
    """Camera-like packets: groups of 64 rays from one origin (a point 8..30 units
    out) into a cone of half-angle `cone` around the direction to a random hair
    vertex -- coherent like a pixel's samples, plus wider cones."""
    rng = np.random.default_rng(seed)
    xyz, _ = r.hair()
    tgt = xyz[rng.integers(0, len(xyz), n_groups)].astype(np.float64)
    q = rng.normal(size=(n_groups, 3))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    orig = tgt + q * rng.uniform(8.0, 30.0, (n_groups, 1))
    c = (tgt - orig) / np.linalg.norm(tgt - orig, axis=1, keepdims=True)
    d = np.repeat(c, 64, 0) + rng.normal(size=(n_groups * 64, 3)) * cone
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(orig, 64, 0).astype(np.float32)
    n = n_groups * 64
    return o, d.astype(np.float32), np.full(n, 1e-4, np.float32), np.full(n, np.inf, np.float32)


@pytest.mark.parametrize("fixture", ["furball", "straight", "haircurl"])
def test_packet_trace_bit_exact(fixture, request):
    """k_trace_packet's traversal (the camera pass) on coherent 64-ray packets
    gives every lane exactly its own Havran traversal's hit."""
    _, r, o = request.getfixturevalue(fixture)
    for cone, seed in ((2e-4, 11), (3e-3, 12), (3e-2, 13)):
        orig, dirs, mint, maxt = _packet_rays(r, 600, seed, cone)
        gt, giv, gp = r.trace(orig, dirs, mint, maxt, packet=True)
        ot, oiv, op = o.trace(orig, dirs, mint, maxt)
        assert (oiv >= 0).sum() > 500
        np.testing.assert_array_equal(giv, oiv)
        np.testing.assert_array_equal(gt, ot)
        np.testing.assert_array_equal(gp, op)


def test_packet_trace_inline_fallback_bit_exact(furball):
    """The batch entry point finishes an overflowing packet lane by lane inside the kernel
    (tracePackets INLINE: the ring stack and ray rows in the packet's LDS, declared with room
    for them, PacketLdsInline).  With the packet stack limited to 1 and 3 entries most packets
    overflow; every lane's hit must still equal the oracle's Havran traversal."""
    _, r, o = furball
    orig, dirs, mint, maxt = _packet_rays(r, 600, 14, 3e-3)
    ot, oiv, op = o.trace(orig, dirs, mint, maxt)
    assert (oiv >= 0).sum() > 500
    try:
        for entries in (1, 3):
            r.set_packet_stack(entries)
            gt, giv, gp = r.trace(orig, dirs, mint, maxt, packet=True)
            np.testing.assert_array_equal(giv, oiv)
            np.testing.assert_array_equal(gt, ot)
            np.testing.assert_array_equal(gp, op)
    finally:
        r.set_packet_stack(0)


@pytest.fixture(scope="module")
def haircurl():
    """models/hair-curl: four hair shapes with their own roughplastic BSDFs
    (and, here, distinct radii so the per-shape radius path is exercised)."""
    xml, r, o = scene_util.make("haircurl_roughplastic", 300, 48, 40, 8, device=0, radii=HAIRCURL_RADII)
    return xml, r, o


@pytest.fixture(scope="module")
def straight_td():
    xml, r, o = scene_util.make("straight_thindielectric", 1500, 48, 40, 8, device=0)
    return xml, r, o


@pytest.fixture(scope="module")
def straight_md():
    xml, r, o = scene_util.make("straight_dielectric", 1500, 48, 40, 8, device=0)
    return xml, r, o


@pytest.fixture(scope="module")
def furball_rp():
    xml, r, o = scene_util.make("furball_roughplastic", 3000, 48, 40, 8, device=0)
    return xml, r, o


def _assert_directions_close(g, o):
    tight = np.all(np.abs(g - o) <= 1e-4 * np.abs(o) + 1e-4, axis=1)
    assert tight.mean() > 0.9995, tight.mean()
    np.testing.assert_allclose(g, o, rtol=0, atol=1e-2)


def _dirs(rng, n):
    v = rng.normal(size=(n, 3))
    return (v / np.linalg.norm(v, axis=1, keepdims=True)).astype(np.float32)


@pytest.mark.parametrize("fixture", ["furball", "straight", "furball_rp", "straight_md", "straight_td"])
def test_bsdf_matches_oracle(fixture, request):
    _, r, o = request.getfixturevalue(fixture)
    rng = np.random.default_rng(7)
    n = 50000
    wi = _dirs(rng, n)
    wo = _dirs(rng, n)
    u = rng.random((n, 2)).astype(np.float32)
    ge, gpdf, gwo, gw, gsp, gt = r.bsdf(wi, wo, u)
    oe, opdf = o.bsdf_eval(wi, wo)
    # Marschner's longitudinal term is exp(-b + logI0(a) - 1/v + ...) with 1/v up to
    # 400 (marschner_diffuse.cpp:364-374): one ulp of log/exp in the ~400-magnitude
    # argument becomes ~2.4e-5 relative in the value, so the bound is 5e-4.
    np.testing.assert_allclose(ge, oe, rtol=5e-4, atol=1e-7)
    np.testing.assert_allclose(gpdf, opdf, rtol=5e-4, atol=1e-7)
    assert np.mean(np.abs(ge - oe) <= 2e-5 * np.abs(oe) + 1e-30) > 0.99
    owo, ow, osp, ot = o.bsdf_sample(wi, u)
    agree = gt == ot
    assert agree.mean() > 0.999
    # the GGX visible-normal inversion (microfacet.h:652-672) divides by A^2 - 1, which
    # amplifies a one-ulp tan/acos difference near |A| = 1: a handful of directions
    # per 1e5 move by up to ~1e-3, everything else agrees to 1e-4
    _assert_directions_close(gwo[agree], owo[agree])
    close = np.all(np.abs(gw - ow) <= 1e-3 * np.abs(ow) + 1e-6, axis=1)
    assert close[agree].mean() > 0.999


@pytest.mark.parametrize("dist", ["beckmann", "ggx", "phong"])
def test_roughplastic_variants_match_oracle(dist):
    """roughplastic over every microfacet distribution, both sampling
    strategies (visible normals / all normals) and the nonlinear diffuse
    variant, including textures > 1 that ensureEnergyConservation rescales.
    Beckmann + visible normals exercises the erf/erfinv Newton inversion
    (microfacet.h:590-647)."""
    _, r, o = scene_util.make("furball_roughplastic", 600, 16, 16, 1, device=0)
    rng = np.random.default_rng(11)
    n = 40000
    wi = _dirs(rng, n)
    wi[: n // 8, :2] *= 1e-3                       # near-normal incidence (thetaI < 1e-4 branches)
    wi[: n // 8] /= np.linalg.norm(wi[: n // 8], axis=1, keepdims=True)
    wo = _dirs(rng, n)
    u = rng.random((n, 2)).astype(np.float32)
    for sv, nl, alpha, dif, spec, eta in [(True, False, 0.2, (0.143016, 0.0156076, 1.8e-5), (1, 1, 1), (1.55, 1.0)),
                                          (False, True, 0.05, (0.8, 0.3, 0.1), (0.5, 0.6, 0.7), (1.49, 1.000277)),
                                          (True, True, 0.45, (1.3, 0.2, 0.4), (1.2, 1.0, 0.9), (1.0, 1.33))]:
        di = {"beckmann": 0, "ggx": 1, "phong": 2}[dist]
        r.set_roughplastic(eta[0], eta[1], di, alpha, sv, nl, dif, spec)
        r.prepare()
        o.set_roughplastic({"eta": np.float32(eta[0]) / np.float32(eta[1]), "distribution": dist, "alpha": alpha,
                            "sample_visible": sv, "nonlinear": nl, "diffuse": dif, "specular": spec})
        ge, gpdf, gwo, gw, gsp, gt = r.bsdf(wi, wo, u)
        oe, opdf = o.bsdf_eval(wi, wo)
        np.testing.assert_allclose(ge, oe, rtol=5e-4, atol=1e-6)
        np.testing.assert_allclose(gpdf, opdf, rtol=5e-4, atol=1e-6)
        assert np.mean(np.abs(ge - oe) <= 2e-5 * np.abs(oe) + 1e-30) > 0.99
        owo, ow, osp, ot = o.bsdf_sample(wi, u)
        agree = gt == ot
        assert agree.mean() > 0.999, (dist, sv, nl)
        _assert_directions_close(gwo[agree], owo[agree])
        close = np.all(np.abs(gw - ow) <= 1e-3 * np.abs(ow) + 1e-6, axis=1)
        assert close[agree].mean() > 0.999, (dist, sv, nl)


def test_hide_emitters_with_pass_through(straight_md):
    """hideEmitters with a BSDF that has an ENull component: a camera path that
    only passed straight through fibers is still 'unscattered' and must not
    see the environment (path.cpp:205, 238-240); after any reflection it must."""
    _, r, o = straight_md
    si = r.info()
    try:
        r.set_integrator(si.max_depth, si.rr_depth, True, True)
        r.prepare()
        o.lib.orc_set_integrator(o.s, si.max_depth, si.rr_depth, 1, 1)
        film = r.render(0, si.spp)
        ofilm, _ = o.render(0, si.spp, width=si.width, height=si.height)
        a, b = native.develop(film), native.develop(ofilm)
        m = scene_util.l2_metrics(b, a)
        print("hideEmitters gpu vs oracle", m)
        assert m["rmse"] < 1e-3, m
        same = np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7, axis=-1)
        assert same.mean() > 0.85
    finally:
        r.set_integrator(si.max_depth, si.rr_depth, True, False)
        r.prepare()
        o.lib.orc_set_integrator(o.s, si.max_depth, si.rr_depth, 1, 0)


def test_envmap_matches_oracle(furball):
    _, r, o = furball
    rng = np.random.default_rng(9)
    n = 30000
    ref = (np.array([0.0, 12.3, 0.0]) + rng.normal(0, 1.0, (n, 3))).astype(np.float32)
    u = rng.random((n, 2)).astype(np.float32)
    dq = _dirs(rng, n)
    gd, gv, gp, gdist, ge, gep = r.env(ref, u, dq)
    od, ov, op, odist = o.env_sample(ref, u)
    np.testing.assert_allclose(gd, od, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(gv, ov, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(gp, op, rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(gdist, odist, rtol=1e-5)
    oe, oep = o.env_eval(dq)
    # atan2/acos ulp differences move the bilinear weights by ~1e-7 x 512 texels; at the
    # sun-disk edge the texel jump (~60) turns that into ~2e-3 absolute.
    np.testing.assert_allclose(ge, oe, rtol=5e-3, atol=2e-3)
    np.testing.assert_allclose(gep, oep, rtol=5e-3, atol=2e-3)
    tight = np.all(np.abs(ge - oe) <= 2e-5 * np.abs(oe) + 1e-7, axis=1)
    assert tight.mean() > 0.995


def test_env_filtered_matches_oracle(furball):
    """Camera-ray environment lookups with ray differentials: EWA over the MIP
    pyramid (mipmap.h:629-834) -- footprints from well below a texel (bilinear at
    level 0) to many levels (trilinear / EWA between levels, the box filter past
    the top), anisotropic up to 100:1 (the maxAnisotropy = 10 clamp)."""
    _, r, o = furball
    rng = np.random.default_rng(21)
    n = 30000
    d = _dirs(rng, n).astype(np.float64)
    t1 = np.cross(d, rng.normal(size=(n, 3)))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    t2 = np.cross(d, t1)
    ang = rng.uniform(0, 2 * np.pi, n)[:, None]
    t1, t2 = np.cos(ang) * t1 + np.sin(ang) * t2, -np.sin(ang) * t1 + np.cos(ang) * t2
    e1 = 10 ** rng.uniform(-4.5, -0.3, n)[:, None]
    e2 = e1 * 10 ** rng.uniform(-2, 0, n)[:, None]
    rx = d + t1 * e1
    ry = d + t2 * e2
    rx /= np.linalg.norm(rx, axis=1, keepdims=True)
    ry /= np.linalg.norm(ry, axis=1, keepdims=True)
    g = r.env_filtered(d, rx, ry)
    oe = o.env_eval_filtered(d, rx, ry)
    assert np.all(np.isfinite(g)) and g.max() > 0
    np.testing.assert_allclose(g, oe, rtol=5e-3, atol=2e-3)
    tight = np.all(np.abs(g - oe) <= 2e-4 * np.abs(oe) + 1e-6, axis=1)
    assert tight.mean() > 0.99, tight.mean()
    # below a texel the filtered lookup is the plain bilinear one
    small = (e1[:, 0] < 1e-4)
    b, _ = o.env_eval(d[small])
    np.testing.assert_allclose(oe[small], b, rtol=1e-6, atol=1e-7)


def test_render_ewa_primary_misses():
    """A coarse frame (24x18, 2 spp) whose camera-ray footprints span ~1.5 texels of
    the sky, so primary misses take the EWA branch (oracle stats[5] counts them);
    the film matches the oracle at the noise floor's level."""
    _, r, o = scene_util.make("furball_marschner", 1500, 24, 18, 2, device=0)
    film = r.render(0, 2)
    ofilm, ostats = o.render(0, 2, width=24, height=18)
    assert int(ostats[5]) > 50, "the EWA branch was not exercised"
    m = scene_util.l2_metrics(native.develop(ofilm), native.develop(film))
    assert m["rel_rmse"] < 1e-3, m


@pytest.mark.parametrize("strands", [[], [[(0.0, 12.0, 0.0)]], [[(0.0, 12.0, 0.0), (0.3, 12.6, 0.1)]]],
                         ids=["empty", "one-vertex", "one-segment"])
def test_render_degenerate_hair(tmp_path, strands):
    """Empty and single-vertex hair files (no segment: the kd-tree is one empty
    leaf, every ray misses -> the sky) and a single segment: GPU film == oracle."""
    import re
    from mitsuba_amd import synth_hair
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=10)
    hair = tmp_path / "h.mitshair"
    synth_hair.write_binary_hair(str(hair), strands)
    src = re.sub(r'value="furball_10\.mitshair"', 'value="h.mitshair"', open(xml).read())
    x2 = tmp_path / "deg.xml"
    x2.write_text(src)
    r = native.Renderer(device=0)
    r.load_scene_xml(str(x2), {"width": 32, "height": 24, "spp": 4})
    r.prepare()
    film = r.render(0, 4)
    _, cam, bsdf = scene_util.config_params("furball_marschner")
    o = oracle_lib.Oracle()
    o.setup(cam, 35.0, 32, 24, str(hair), float(scene_util.scenes.CONFIGS["furball_marschner"]["radius"]), bsdf,
            scene_util.oracle_envmap("furball_marschner"), 65, spp=4)
    nodes, idx, _ = r.kdtree()
    o.set_kdtree(nodes, idx)
    o.prepare()
    ofilm, _ = o.render(0, 4, width=32, height=24)
    assert np.all(np.isfinite(film)) and film[..., 3].sum() > 0
    m = scene_util.l2_metrics(native.develop(ofilm), native.develop(film))
    assert m["rel_rmse"] < 1e-4, m


def _reference_flags_floor(fixture, r, si):
    name, n = {"furball": ("furball_marschner", 3000), "straight": ("straight_kk", 1500),
               "furball_rp": ("furball_roughplastic", 3000), "straight_md": ("straight_dielectric", 1500),
               "straight_td": ("straight_thindielectric", 1500), "haircurl": ("haircurl_roughplastic", 300)}[fixture]
    return scene_util.reference_flags_floor(name, n, r, si.width, si.height, si.spp,
                                            radii=HAIRCURL_RADII if fixture == "haircurl" else None)


@pytest.mark.parametrize("fixture", ["furball", "straight", "furball_rp", "straight_md", "straight_td", "haircurl"])
def test_render_matches_oracle(fixture, request):
    """Full wavefront render vs the oracle's MIPathTracer::Li restatement."""
    _, r, o = request.getfixturevalue(fixture)
    si = r.info()
    film = r.render(0, si.spp, collect_stats=2)
    ofilm, ostats = o.render(0, si.spp, width=si.width, height=si.height)
    assert int(ostats[5]) == 0, "EWA lookups that do not reduce to bilinear"
    # the sample weights are identical bit for bit up to summation order
    np.testing.assert_allclose(film[..., 3], ofilm[..., 3], rtol=1e-5)
    a = native.develop(film)
    b = native.develop(ofilm)
    m = scene_util.l2_metrics(b, a)
    # Most paths are bit-identical; a path diverges only when a one-ulp difference
    # of a float32 transcendental (ocml vs glibc) flips a discrete decision (grazing
    # hair hit, lobe choice, Russian roulette).  Such a path changes its pixel by
    # O(radiance / spp), so at 8 spp the bound is on the absolute per-pixel RMSE
    # (north_star: < 1e-3, linear HDR units) plus the fraction of exact pixels.
    same = np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7, axis=-1)
    # Noise floor: the same oracle compiled with the reference's own flags
    # (-funsafe-math-optimizations, config-ubuntu-20.04.py:8) vs the strict build.
    floor, floor_same = _reference_flags_floor(fixture, r, si)
    print(fixture, "gpu vs oracle", m, "identical %.4f" % same.mean(), "| floor", floor, "identical %.4f" % floor_same)
    scene_util.assert_at_floor(m, floor, same.mean(), floor_same, factor=2.0)
    s = r.stats()
    assert s.paths == si.width * si.height * si.spp or s.paths >= si.width * si.height * si.spp
    assert s.nodes + s.packet_nodes > 0 and s.prims + s.packet_prims > 0
    assert s.trace_launches + s.packet_launches >= 1
    assert s.trace_launches >= 1 or s.tail_paths > 0  # later bounces ran per launch or in k_tail


def test_render_deterministic_and_sharded(furball):
    _, r, o = furball
    si = r.info()
    a = r.render(0, si.spp)
    b = r.render(0, si.spp)
    np.testing.assert_array_equal(a, b)
    # two shards of 32x32 blocks summed == the full frame (up to summation order)
    s = r.render(0, si.spp, shard=0, n_shards=2)
    s = r.render(0, si.spp, shard=1, n_shards=2, film=s)
    np.testing.assert_allclose(s, a, rtol=1e-5, atol=1e-6)
    # spp ranges accumulate: [0, 3) + [3, spp) == [0, spp)
    c = r.render(0, 3)
    c = r.render(3, si.spp, film=c)
    np.testing.assert_allclose(c, a, rtol=1e-5, atol=1e-6)
    # small waves give the same result as one wave
    d = r.render(0, si.spp, max_wave_paths=4096)
    np.testing.assert_allclose(d, a, rtol=1e-5, atol=1e-6)
    # each shard renders exactly the blocks distributed.block_owner deals it
    W, H = si.width, si.height
    nbx, nby = (W + 31) // 32, (H + 31) // 32
    for n_shards in (2, 3):
        owner = distributed.block_owner(nbx, nby, n_shards)
        for shard in range(n_shards):
            f = r.render(0, 2, shard=shard, n_shards=n_shards)
            for b, o_ in enumerate(owner):
                bx, by = b % nbx, b // nbx
                core = f[by * 32 + 1:min(H, by * 32 + 31), bx * 32 + 1:min(W, bx * 32 + 31), 3]
                assert (core.min() > 0) if o_ == shard else (core.max() == 0), (n_shards, shard, b)


@pytest.mark.parametrize("name,n,radii", [("furball_marschner", 1500, None), ("straight_kk", 400, None),
                                          ("haircurl_roughplastic", 300, HAIRCURL_RADII)])
def test_tail_kernel_bit_identical(name, n, radii, monkeypatch):
    """k_tail (every remaining bounce of the few live paths in one launch)
    runs the wavefront kernels' own per-path steps in the same order, so the
    film is bit-identical to per-bounce launches, whichever bounce the tail
    starts at (HPT_TAIL_PATHS: 0 = never, 1<<30 = right after the camera pass,
    default = once fewer than 2^17 paths are live)."""
    films = []
    for tail in ("0", "2000", "1073741824"):
        monkeypatch.setenv("HPT_TAIL_PATHS", tail)
        _, r, _ = scene_util.make(name, n, 64, 48, 16, device=0, radii=radii)
        films.append(r.render(0, 16, collect_stats=True))
        s = r.stats()
        assert (s.tail_paths > 0) == (tail != "0"), (tail, s.tail_paths)
        r.close()
    np.testing.assert_array_equal(films[0], films[1])
    np.testing.assert_array_equal(films[0], films[2])


@pytest.mark.parametrize("spp", [128, 256, 512])
def test_camera_quadrant_packets(spp, monkeypatch):
    """A wave holding 128 / 256 / 512 samples of a pixel queues them by the
    quadrant of the pixel they fall in (k_camera's qpushCamera), so a 64-ray
    packet covers part of the pixel.  Only the queue order changes: the film
    equals the one-ray-per-lane camera pass (HPT_PACKETS=0) bit for bit, and
    the same frame in waves of 64 samples (no reordering) up to summation order;
    at 256 spp it also matches the oracle at the reference-flags floor."""
    films = []
    for packets in ("1", "0"):
        monkeypatch.setenv("HPT_PACKETS", packets)
        _, r, o = scene_util.make("furball_marschner", 3000, 48, 32, spp, device=0)
        films.append(r.render(0, spp, collect_stats=True))
        if packets == "1":
            assert r.stats().packet_launches >= 1
            small = r.render(0, spp, max_wave_paths=2 * 1024 * 64)  # two 32x32 blocks of slots
    np.testing.assert_array_equal(films[0], films[1])
    np.testing.assert_allclose(small, films[0], rtol=1e-5, atol=1e-6)
    if spp == 256:
        ofilm, _ = o.render(0, spp, threads=16, width=48, height=32)
        np.testing.assert_allclose(films[0][..., 3], ofilm[..., 3], rtol=1e-5)
        a, b = native.develop(films[0]), native.develop(ofilm)
        m = scene_util.l2_metrics(b, a)
        same = np.all(np.abs(a - b) <= 1e-5 * np.abs(b) + 1e-7, axis=-1)
        floor, floor_same = scene_util.reference_flags_floor("furball_marschner", 3000, r, 48, 32, spp)
        scene_util.assert_at_floor(m, floor, same.mean(), floor_same, factor=2.0)


def test_full_size_headline_frame():
    """BASELINE.json configs[2] at its full size (furball, 40,000 strands,
    512x512 @ 256 spp, maxDepth 65): deterministic, shard- and spp-split
    invariant; and at full resolution with 64 spp the film matches the
    oracle at the reference-flags noise floor."""
    xml, r, o = scene_util.make("furball_marschner", 40000, 512, 512, 256, device=0)
    a = r.render(0, 256)
    np.testing.assert_array_equal(a, r.render(0, 256))
    s = r.render(0, 256, shard=0, n_shards=3)
    s = r.render(0, 256, shard=1, n_shards=3, film=s)
    s = r.render(0, 256, shard=2, n_shards=3, film=s)
    np.testing.assert_allclose(s, a, rtol=1e-5, atol=1e-5)
    c = r.render(0, 100)
    c = r.render(100, 256, film=c)
    np.testing.assert_allclose(c, a, rtol=1e-5, atol=1e-5)
    img = native.develop(a)
    assert np.all(np.isfinite(img)) and img.mean() > 0
    # full-resolution parity at 64 spp: one flipped discrete event (a path that
    # reaches the sun on one side only) moves a pixel by O(sun radiance / spp),
    # so the film is compared where such flips are averaged like the headline's
    g = native.develop(r.render(0, 64))
    of, ostats = o.render(0, 64, threads=16, width=512, height=512)
    b = native.develop(of)
    m = scene_util.l2_metrics(b, g)
    floor, floor_same = scene_util.reference_flags_floor("furball_marschner", 40000, r, 512, 512, 64)
    same = np.all(np.abs(g - b) <= 1e-5 * np.abs(b) + 1e-7, axis=-1)
    print("full-size gpu vs oracle", m, "identical %.4f" % same.mean(), "| floor", floor, "identical %.4f" % floor_same)
    scene_util.assert_at_floor(m, floor, same.mean(), floor_same, factor=3.0)


def test_cli_renders_and_develops(tmp_path):
    """bin/mitsuba (mitsuba.cpp:52-400 options) on a scene: -D defines, -o with a
    wrong extension (the ldrfilm replaces it), -x skip; the PNG equals the film
    developed through hpt_write_film from a library render of the same scene."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import film as ref
    root = os.path.dirname(native.__file__)
    cli = os.path.join(root, "..", "bin", "mitsuba")
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=800)
    cmd = [cli, "-D", "spp=4", "-D", "width=64", "-D", "height=48", "-o", str(tmp_path / "out.jpg"), xml]
    res = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    png = tmp_path / "out.png"
    assert png.exists()
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"spp": 4, "width": 64, "height": 48})
    r.prepare()
    film = r.render(0, 4)
    out = r.write_film(tmp_path / "lib.png", film)
    np.testing.assert_array_equal(ref.read_png(str(png)), ref.read_png(out))
    res = subprocess.run(cmd + ["-x"], capture_output=True, text=True, timeout=300)
    assert res.returncode == 0 and "Skipping" in res.stdout
    # -r sec: partial images between sample chunks (spp/16 each); the final image is the
    # chunk-accumulated film, as a library render of the same chunks develops it
    cmd_r = [cli, "-D", "spp=32", "-D", "width=64", "-D", "height=48", "-r", "1e-9", "-o",
             str(tmp_path / "part.png"), xml]
    res = subprocess.run(cmd_r, capture_output=True, text=True, timeout=300)
    assert res.returncode == 0, res.stderr
    assert res.stdout.count("Wrote partial image") == 15, res.stdout
    r2 = native.Renderer(device=0)
    r2.load_scene_xml(xml, {"spp": 32, "width": 64, "height": 48})
    r2.prepare()
    f2 = None
    for j0 in range(0, 32, 2):
        f2 = r2.render(j0, j0 + 2, film=f2)
    out2 = r2.write_film(tmp_path / "lib2.png", f2)
    np.testing.assert_array_equal(ref.read_png(str(tmp_path / "part.png")), ref.read_png(out2))


def test_sobol_scramble_render(tmp_path):
    """SobolSampler 'scramble' (sobol.cpp:92-102): TEA of the property, XORed
    into every sample and into the pixel look-up (sobolseq.h:43-58, 99-131)."""
    xml, r, o = scene_util.make("straight_kk", 800, 40, 32, 4, device=0)
    src = open(xml).read().replace('<integer name="sampleCount" value="$spp"/>',
                                   '<integer name="sampleCount" value="$spp"/><integer name="scramble" value="987654321987"/>')
    path = tmp_path / "scr.xml"
    path.write_text(src.replace('value="straight_', 'value="' + scene_util.WORK + '/straight_'))
    r2 = native.Renderer(device=0)
    r2.load_scene_xml(str(path), {"width": 40, "height": 32, "spp": 4})
    r2.prepare()
    o.check(o.lib.orc_set_sobol_scramble(o.s, 987654321987))
    rng = np.random.default_rng(2)
    n = 5000
    frame = rng.integers(0, 64, n).astype(np.uint32)
    px = rng.integers(0, 32, n).astype(np.uint32)
    py = rng.integers(0, 32, n).astype(np.uint32)
    dim = rng.integers(0, 300, n).astype(np.uint32)
    gi, gv = r2.sobol(6, frame, px, py, dim)
    oi = o.sobol_lookup(6, frame, px, py)
    np.testing.assert_array_equal(gi, oi)
    np.testing.assert_array_equal(gv, o.sobol_sample(oi, dim))
    gi0, _ = r.sobol(6, frame, px, py, dim)
    assert np.mean(gi0 != gi) > 0.5  # the scramble changes the sample set
    film = r2.render(0, 4)
    ofilm, _ = o.render(0, 4, width=40, height=32)
    m = scene_util.l2_metrics(native.develop(ofilm), native.develop(film))
    assert m["rmse"] < 1e-3, m
    o.check(o.lib.orc_set_sobol_scramble(o.s, 0))
