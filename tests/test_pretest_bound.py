"""The 16-byte pre-test record (HptSegQ, hpt_device.h) stays conservative.

k_trace's leaf pass rejects a segment when the ray line passes farther than
`preRadius` from the line through v1 along the *oct-quantised* axis
(segMayHitQ, hpt_render.hip).  kdtree_build.cpp sets preRadius to
max_s r_s + reach_s * sin(theta_s): a point the exact test accepts (hair.cpp:
485-548: inside the cylinder and between the two miter planes) lies at an
axial offset s in [-r tan(phi1), len + r tan(phi2)] from v1, so within
r + |s| sin(theta) of the quantised line.  This test restates the encode /
decode and the bound in numpy (fp32 where the device computes in fp32) and
checks, on rays aimed at points just inside random mitered cylinders (grazing
and head-on), that every ray the fp64 exact test accepts passes the quantised
fp32 pre-test.  The GPU side of the same property is the bit-exact trace
tests (tests/test_gpu_parity.py: mixed and grazing rays against the oracle).
"""
import numpy as np

F = np.float32


def oct_encode(a):
    """kdtree_build.cpp axisOctEncode: fp64 axis -> 16:16 bits."""
    l1 = np.abs(a).sum(axis=1)
    u, v = a[:, 0] / l1, a[:, 1] / l1
    neg = a[:, 2] < 0
    fu = (1.0 - np.abs(v)) * np.where(u >= 0, 1.0, -1.0)
    fv = (1.0 - np.abs(u)) * np.where(v >= 0, 1.0, -1.0)
    u, v = np.where(neg, fu, u), np.where(neg, fv, v)
    q = lambda x: np.clip(np.rint((x * 0.5 + 0.5) * 65535.0), 0, 65535).astype(np.uint32)  # noqa: E731
    return q(u) | (q(v) << 16)


def oct_decode(q):
    """axisOctDecode (device and host): fp32 operations."""
    k = F(2.0) / F(65535.0)
    u = (q & 0xFFFF).astype(F) * k - F(1)
    v = (q >> 16).astype(F) * k - F(1)
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
