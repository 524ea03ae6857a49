"""The 16-byte pre-test record (HptSegQ, hpt_device.h) stays conservative, per record.

k_trace's leaf pass rejects a segment when the ray line passes farther than the
scene's pre-test radius from the line through v1 along the *oct-quantised* axis
(segMayHitQ, hpt_render.hip), unless the record is flagged to pass.  A point the exact test accepts (hair.cpp:
485-548: inside the cylinder and between the two miter planes) lies at an
axial offset s in [-r tan(phi1), len + r tan(phi2)] from v1, so within
r + |s| sin(theta) of the quantised line: that is the record's bound
(kdtree_build.cpp quantisedReach).  A record whose bound exceeds its shape's
radius by more than 5 % (a fold) is flagged to pass every pre-test, and the
scene's radius is the largest bound of the others, so a fold no longer widens
the test of every record.  This test restates the encode /
decode and the bound in numpy (fp32 where the device computes in fp32) and
checks, on rays aimed at points just inside random mitered cylinders (grazing
and head-on), that every ray the fp64 exact test accepts passes the quantised
fp32 pre-test; then the same on the library's own records of a furball with
folded strands (scene_util.fold_workdir: an exact hairpin, a near-exact fold,
a 179.9 degree fold), whose folds must not widen the other records' test.
The GPU side of the same property is the bit-exact trace tests
(tests/test_gpu_parity.py: mixed and grazing rays against the oracle) and
tests/test_gpu_configs.py's fold scene.
"""
import numpy as np
import pytest

import scene_util
from mitsuba_amd import native

F = np.float32


def oct_encode(a):
    """kdtree_build.cpp axisOctEncode: fp64 axis -> u 16 bits, v 15 bits (bit 31: the pass flag)."""
    l1 = np.abs(a).sum(axis=1)
    u, v = a[:, 0] / l1, a[:, 1] / l1
    neg = a[:, 2] < 0
    fu = (1.0 - np.abs(v)) * np.where(u >= 0, 1.0, -1.0)
    fv = (1.0 - np.abs(u)) * np.where(v >= 0, 1.0, -1.0)
    u, v = np.where(neg, fu, u), np.where(neg, fv, v)
    q = lambda x, m: np.clip(np.rint((x * 0.5 + 0.5) * m), 0, m).astype(np.uint32)  # noqa: E731
    return q(u, 65535.0) | (q(v, 32767.0) << 16)


def oct_decode(q):
    """axisOctDecode (device and host): fp32 operations."""
    u = (q & 0xFFFF).astype(F) * (F(2.0) / F(65535.0)) - F(1)
    v = ((q >> 16) & 0x7FFF).astype(F) * (F(2.0) / F(32767.0)) - F(1)
    z = F(1) - np.abs(u) - np.abs(v)
    fx = (F(1) - np.abs(v)) * np.where(u >= 0, F(1), F(-1))
    fy = (F(1) - np.abs(u)) * np.where(v >= 0, F(1), F(-1))
    neg = z < 0
    return np.stack([np.where(neg, fx, u), np.where(neg, fy, v), z], axis=1).astype(F)


def unit(x):
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def test_oct_roundtrip_angle_small():
    rng = np.random.default_rng(3)
    a = unit(rng.normal(size=(100000, 3)))
    a[:6] = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [-1, 0, 0], [0, -1, 0], [0, 0, -1]]
    q = oct_decode(oct_encode(a)).astype(np.float64)
    sin_t = np.linalg.norm(np.cross(a, q), axis=1) / np.linalg.norm(q, axis=1)
    assert sin_t.max() < 1e-4  # 16-bit oct cells: a few 1e-5 rad
    assert np.all(np.linalg.norm(q, axis=1) >= 1 / np.sqrt(3) - 1e-6)


def test_quantised_pretest_is_conservative():
    rng = np.random.default_rng(7)
    n = 200000
    v1 = rng.uniform(-1, 1, size=(n, 3)).astype(F).astype(np.float64)  # hair vertices are fp32
    a = unit(rng.normal(size=(n, 3)))
    length = rng.uniform(0.005, 0.3, size=n)
    v2 = v1 + a * length[:, None]
    r = np.full(n, F(0.004), dtype=np.float64)  # one hair shape

    def bisector(max_deg):
        # miter normal: the bisector of the axis and a neighbour direction turned by up to max_deg
        t = unit(np.cross(a, rng.normal(size=(n, 3))))
        ang = np.radians(rng.uniform(0, max_deg, size=n))[:, None]
        nb = a * np.cos(ang) + t * np.sin(ang)
        return unit(nb + a)

    n1, n2 = bisector(80.0), bisector(80.0)
    # kdtree_build.cpp quantisedReach + the 1e-5 slack
    q = oct_encode(a)
    qa = oct_decode(q)
    qd = qa.astype(np.float64)
    sin_t = np.linalg.norm(np.cross(a, qd), axis=1) / np.linalg.norm(qd, axis=1)
    tan_of = lambda nn: np.sqrt(np.maximum(0, 1 - np.sum(nn * a, 1) ** 2)) / np.abs(np.sum(nn * a, 1))  # noqa: E731
    reach = np.maximum(r * tan_of(n1), length + r * tan_of(n2))
    pre_r = np.float32(np.max(r + reach * sin_t) * (1 + 1e-5))

    # a target point just inside the mitered cylinder, the ray through it from a random direction
    lo, hi = -r * tan_of(n1), length + r * tan_of(n2)
    s = lo + (hi - lo) * rng.uniform(size=n)
    perp = unit(np.cross(a, rng.normal(size=(n, 3))))
    p = v1 + a * s[:, None] + perp * (r * (1 - 10 ** rng.uniform(-9, -3, size=n)))[:, None]
    grazing = rng.uniform(size=n) < 0.5
    d = unit(np.where(grazing[:, None], np.cross(a, perp) + 0.05 * rng.normal(size=(n, 3)), rng.normal(size=(n, 3))))
    d = d.astype(F)
    # origins close to the segment keep the fp32 rounding margin (3e-6 |w|) below the quantisation's turn
    o = (p - d.astype(np.float64) * rng.uniform(0.01, 0.2, size=n)[:, None]).astype(F)

    # fp64 exact test (hair.cpp:485-548): cylinder roots, then the miter planes
    od, dd = o.astype(np.float64), d.astype(np.float64)
    rel = od - v1
    po = rel - a * np.sum(a * rel, 1)[:, None]
    pd = dd - a * np.sum(a * dd, 1)[:, None]
    A, B, C = np.sum(pd * pd, 1), 2 * np.sum(po * pd, 1), np.sum(po * po, 1) - r * r
    disc = B * B - 4 * A * C
    ok = (A > 0) & (disc >= 0)
    sq = np.sqrt(np.maximum(disc, 0))
    hit = np.zeros(n, bool)
    for sign in (-1.0, 1.0):
        t = np.where(ok, (-B + sign * sq) / np.where(A > 0, 2 * A, 1), np.nan)
        x = od + dd * t[:, None]
        inside = (np.sum((x - v1) * n1, 1) >= 0) & (np.sum((x - v2) * n2, 1) <= 0) & (t > 0)
        hit |= ok & inside
    assert hit.sum() > n // 4

    # the device pre-test (segMayHit on the decoded axis), fp32 without contraction
    w = o - v1.astype(F)
    ax, ay, az = qa[:, 0], qa[:, 1], qa[:, 2]
    nx = d[:, 1] * az - d[:, 2] * ay
    ny = d[:, 2] * ax - d[:, 0] * az
    nz = d[:, 0] * ay - d[:, 1] * ax
    nn = nx * nx + ny * ny + nz * nz
    wn = np.abs(w[:, 0] * nx + w[:, 1] * ny + w[:, 2] * nz)
    margin = F(3e-6) * (pre_r + np.abs(w[:, 0]) + np.abs(w[:, 1]) + np.abs(w[:, 2]))
    may = wn <= pre_r * np.sqrt(nn) * F(1.000001) + margin
    assert not np.any(hit & ~may), "quantised pre-test rejected %d exact hits" % np.sum(hit & ~may)


def exact_hits(o, d, v1, v2, a, n1, n2, r):
    """fp64 exact test (hair.cpp:485-548): cylinder roots, then the miter planes (NaN-aware like
    the reference: a NaN plane test fails)."""
    od, dd = o.astype(np.float64), d.astype(np.float64)
    rel = od - v1
    po = rel - a * np.sum(a * rel, 1)[:, None]
    pd = dd - a * np.sum(a * dd, 1)[:, None]
    A, B, C = np.sum(pd * pd, 1), 2 * np.sum(po * pd, 1), np.sum(po * po, 1) - r * r
    disc = B * B - 4 * A * C
    ok = (A > 0) & (disc >= 0)
    sq = np.sqrt(np.maximum(disc, 0))
    hit = np.zeros(len(o), bool)
    with np.errstate(invalid="ignore"):
        for sign in (-1.0, 1.0):
            t = np.where(ok, (-B + sign * sq) / np.where(A > 0, 2 * A, 1), np.nan)
            x = od + dd * t[:, None]
            inside = (np.sum((x - v1) * n1, 1) >= 0) & (np.sum((x - v2) * n2, 1) <= 0) & (t > 0)
            hit |= ok & inside
    return hit


def pretest(o, d, v1f, qa, rad):
    """segMayHit on the decoded axis qa at radius rad (per record), fp32 without contraction."""
    w = o - v1f
    ax, ay, az = qa[:, 0], qa[:, 1], qa[:, 2]
    nx = d[:, 1] * az - d[:, 2] * ay
    ny = d[:, 2] * ax - d[:, 0] * az
    nz = d[:, 0] * ay - d[:, 1] * ax
    nn = nx * nx + ny * ny + nz * nz
    wn = np.abs(w[:, 0] * nx + w[:, 1] * ny + w[:, 2] * nz)
    margin = F(3e-6) * (rad + np.abs(w[:, 0]) + np.abs(w[:, 1]) + np.abs(w[:, 2]))
    return wn <= rad * np.sqrt(nn) * F(1.000001) + margin


def _segments(r):
    """Per leaf entry of the library's kd-tree: fp64 v1, v2, axis, miter normals (hair.cpp:551-596)
    from its own merged vertices, and the record words."""
    xyz, starts = r.hair()
    _, iv, _ = r.kdtree()
    iv = iv.astype(np.int64)
    rec, radius, n_pass = r.pretest_records()
    assert rec.shape == (len(iv), 4)
    X = xyz.astype(np.float64)

    def nrm(x):
        with np.errstate(invalid="ignore", divide="ignore"):
            return x / np.linalg.norm(x, axis=1, keepdims=True)

    v1, v2 = X[iv], X[iv + 1]
    a = nrm(v2 - v1)
    has_prev, has_next = starts[iv] == 0, starts[iv + 2] == 0
    n1 = np.where(has_prev[:, None], nrm(nrm(v1 - X[np.maximum(iv - 1, 0)]) + a), a)
    n2 = np.where(has_next[:, None], nrm(a + nrm(X[np.minimum(iv + 2, len(X) - 1)] - v2)), a)
    return v1, v2, a, n1, n2, rec, radius, n_pass


def _fold_renderer(folded):
    d = scene_util.fold_workdir(3000, folded)
    xml = scene_util.scenes.make_scene("furball_marschner", d, n_strands=3000)
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(xml, {"width": 64, "height": 64, "spp": 4})
    r.prepare()
    return r


@pytest.fixture(scope="module")
def fold_scene():
    r = _fold_renderer(True)
    yield r
    r.close()


def test_library_records_match_the_restatement(fold_scene):
    # the library's axis bits are numpy's oct_encode of the fp64 axis, v1 its fp32 first vertex
    v1, _, a, _, _, rec, _, _ = _segments(fold_scene)
    np.testing.assert_array_equal(rec[:, 3] & 0x7FFFFFFF, oct_encode(a))
    np.testing.assert_array_equal(rec[:, :3].view(np.float32), v1.astype(np.float32))


def test_fold_records_pass_without_widening(fold_scene):
    v1, v2, a, n1, n2, rec, radius, n_pass = _segments(fold_scene)
    rad = F(0.00216667)
    flag = (rec[:, 3] >> 31).astype(bool)
    with np.errstate(invalid="ignore"):
        folded = (np.abs(np.sum(n1 * a, 1)) < 0.01) | (np.abs(np.sum(n2 * a, 1)) < 0.01)
    nan_normal = np.isnan(n1).any(1) | np.isnan(n2).any(1)
    # the near-hairpin (a bound of ~150 radii) is flagged, and only a fold is: the radius every
    # other record is tested at stays within 5 % of the shape's (the 179.9 degree fold's bound)
    assert n_pass == flag.sum() and 0 < n_pass <= 8, n_pass
    assert np.all(folded[flag]), "an unfolded record is flagged"
    assert rad <= radius < 1.05 * rad, radius
    # the exact hairpin's NaN miter normals: no exact test accepts the segment, it needs no flag
    assert nan_normal.sum() >= 2 and not np.any(flag[nan_normal])


def test_per_record_pretest_is_conservative(fold_scene):
    """Rays aimed just inside each record's mitered cylinder -- every fold record and a sample of
    the rest -- pass k_trace's pre-test (the scene's radius, or the flag) whenever the exact test
    hits; without its flag the near-hairpin's exact hits would be rejected."""
    v1, v2, a, n1, n2, rec, radius, _ = _segments(fold_scene)
    flag = (rec[:, 3] >> 31).astype(bool)
    rng = np.random.default_rng(11)
    qa = oct_decode(rec[:, 3])
    rad = 0.00216667
    ok = ~(np.isnan(n1).any(1) | np.isnan(n2).any(1))
    with np.errstate(invalid="ignore"):
        folded = (np.abs(np.sum(n1 * a, 1)) < 0.01) | (np.abs(np.sum(n2 * a, 1)) < 0.01)
    wide = np.nonzero(ok & folded)[0]
    rest = rng.choice(np.nonzero(ok)[0], 4000, replace=False)
    e = np.concatenate([np.repeat(wide, 4000), np.repeat(rest, 20)])
    n = len(e)
    A, V1, V2, N1, N2 = a[e], v1[e], v2[e], n1[e], n2[e]
    r = np.full(n, float(F(rad)))
    length = np.linalg.norm(V2 - V1, axis=1)
    cos1, cos2 = np.abs(np.sum(N1 * A, 1)), np.abs(np.sum(N2 * A, 1))
    tan1 = np.sqrt(np.maximum(0, 1 - cos1 ** 2)) / cos1
    tan2 = np.sqrt(np.maximum(0, 1 - cos2 ** 2)) / cos2
    # target points over the whole accepted axial range, the far ends of a fold's wedge included
    lo, hi = -r * tan1, length + r * tan2
    s = lo + (hi - lo) * rng.uniform(size=n) ** np.where(rng.uniform(size=n) < 0.5, 1.0, 0.2)
    perp = np.cross(A, rng.normal(size=(n, 3)))
    perp /= np.linalg.norm(perp, axis=1, keepdims=True)
    p = V1 + A * s[:, None] + perp * (r * (1 - 10 ** rng.uniform(-9, -3, size=n)))[:, None]
    dd = np.where((rng.uniform(size=n) < 0.5)[:, None], np.cross(A, perp) + 0.05 * rng.normal(size=(n, 3)),
                  rng.normal(size=(n, 3)))
    d = (dd / np.linalg.norm(dd, axis=1, keepdims=True)).astype(F)
    o = (p - d.astype(np.float64) * rng.uniform(0.01, 0.2, size=n)[:, None]).astype(F)
    hit = exact_hits(o, d, V1, V2, A, N1, N2, r)
    assert hit[: len(wide) * 4000].sum() > 1000 and hit.sum() > n // 5
    test = pretest(o, d, V1.astype(F), qa[e], np.full(n, F(radius)))
    may = test | flag[e]
    assert not np.any(hit & ~may), "pre-test rejected %d exact hits" % np.sum(hit & ~may)
    assert np.any(hit & ~test), "no flagged record needed its flag"


def test_fold_free_twin_radius():
    r = _fold_renderer(False)
    _, _, _, _, _, rec, radius, n_pass = _segments(r)
    assert radius < 1.02 * 0.00216667 and n_pass == 0, (radius, n_pass)
    r.close()
