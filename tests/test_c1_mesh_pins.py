"""Independent pins of the oracle's C1 mesh restatement (oracle/mesh_bsdf.h, mesh_geom.h).

Each check restates the reference formula again in float64 numpy (or uses
scipy's quadrature) and compares with the oracle's float32 code:

  fresnelDiffuseReflectance   util.cpp:808-859 (Lobatto of fresnelDielectricExt(sqrt(xi)))
  SmoothPlastic eval / pdf    plastic.cpp:245-307, sample :372-417
  TwoSidedBRDF                twosided.cpp:108-183
  Checkerboard + Texture2D    checkerboard.cpp:65-73, texture.cpp:112-121
  TriAccel                    triaccel.h:61-158 against a float64 Moller-Trumbore
  OBJ face forms              obj.cpp:244-334, 371-390, 608-715 (fan, negative indices, a//c,
                              a/b, flipTexCoords, vertex merging), faceNormals / flipNormals
                              (trimesh.cpp:608-681), Rectangle (rectangle.cpp:80-168)
CPU only.
"""
import os

import numpy as np
import pytest
from scipy import integrate

import oracle_lib


def fresnel_ext(cos_i, eta):
    """util.cpp:651-681 in float64."""
    if eta == 1:
        return 0.0
    scale = 1 / eta if cos_i > 0 else eta
    ct2 = 1 - (1 - cos_i * cos_i) * scale * scale
    if ct2 <= 0:
        return 1.0
    ci, ct = abs(cos_i), np.sqrt(ct2)
    rs = (ci - eta * ct) / (ci + eta * ct)
    rp = (eta * ci - ct) / (eta * ci + ct)
    return 0.5 * (rs * rs + rp * rp)


def fdr64(eta):
    return integrate.quad(lambda xi: fresnel_ext(np.sqrt(xi), eta), 0, 1, epsabs=1e-12, limit=200)[0]


@pytest.mark.parametrize("eta", [1.5, 1 / 1.5, 1.33, 1 / 1.33, 2.0])
def test_fresnel_diffuse_reflectance(eta):
    got = oracle_lib.fresnel_diffuse_reflectance(np.float32(eta))
    assert abs(got - fdr64(np.float32(eta))) < 2e-5


def _dirs(rng, n, upper=True):
    v = rng.normal(size=(n, 3))
    v /= np.linalg.norm(v, axis=1, keepdims=True)
    if upper:
        v[:, 2] = np.abs(v[:, 2]) + 1e-3
        v /= np.linalg.norm(v, axis=1, keepdims=True)
    return v.astype(np.float32)


def _plastic_oracle(eta=1.5, nonlinear=True, diffuse=(0.9, 0.9, 0.9), specular=(1, 1, 1), ensure=True):
    o = oracle_lib.MeshOracle()
    o.new_bsdf({"type": "plastic", "intIOR": eta, "extIOR": 1.0, "nonlinear": nonlinear, "diffuse": diffuse,
                "specular": specular, "ensureEnergyConservation": ensure})
    return o


def _plastic64(wi, wo, eta, nonlinear, diffuse, specular):
    fdr_int = fdr64(1 / eta)
    lum = lambda c: 0.212671 * c[0] + 0.715160 * c[1] + 0.072169 * c[2]
    sw = lum(specular) / (lum(diffuse) + lum(specular))
    out, pdf = np.zeros((len(wi), 3)), np.zeros(len(wi))
    d = np.array(diffuse, float)
    diff = d / (1 - d * fdr_int) if nonlinear else d / (1 - fdr_int)
    for k, (a, b) in enumerate(zip(wi.astype(float), wo.astype(float))):
        if a[2] <= 0 or b[2] <= 0:
            continue
        fi, fo = fresnel_ext(a[2], eta), fresnel_ext(b[2], eta)
        out[k] = diff * (b[2] / np.pi / eta ** 2 * (1 - fi) * (1 - fo))
        ps = fi * sw / (fi * sw + (1 - fi) * (1 - sw))
        pdf[k] = b[2] / np.pi * (1 - ps)
    return out, pdf


@pytest.mark.parametrize("nonlinear", [True, False])
def test_plastic_eval_pdf(nonlinear):
    rng = np.random.default_rng(5)
    wi, wo = _dirs(rng, 400), _dirs(rng, 400)
    wo[::7, 2] *= -1  # below the surface: zero
    diffuse, specular = (0.9, 0.5, 0.2), (1.0, 0.8, 0.9)
    o = _plastic_oracle(1.5, nonlinear, diffuse, specular)
    rgb, pdf = o.bsdf_eval(wi, wo)
    e_rgb, e_pdf = _plastic64(wi, wo, np.float32(1.5), nonlinear, diffuse, specular)
    np.testing.assert_allclose(rgb, e_rgb, rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(pdf, e_pdf, rtol=2e-5, atol=1e-7)


@pytest.mark.parametrize("ensure", [True, False])
def test_plastic_energy_conservation(ensure):
    """BSDF::ensureEnergyConservation (bsdf.cpp:88-113): a reflectance above 1 is scaled by
    0.99 / max -- unless the BSDF sets ensureEnergyConservation=false"""
    rng = np.random.default_rng(9)
    wi, wo = _dirs(rng, 200), _dirs(rng, 200)
    diffuse, specular = (1.2, 0.6, 0.3), (1.0, 1.0, 1.0)
    rgb, pdf = _plastic_oracle(1.5, False, diffuse, specular, ensure).bsdf_eval(wi, wo)
    d_eff = np.array(diffuse) * (0.99 / 1.2 if ensure else 1.0)
    e_rgb, e_pdf = _plastic64(wi, wo, np.float32(1.5), False, tuple(d_eff), specular)
    np.testing.assert_allclose(rgb, e_rgb, rtol=2e-5, atol=1e-7)
    np.testing.assert_allclose(pdf, e_pdf, rtol=2e-5, atol=1e-7)


def test_plastic_sample():
    rng = np.random.default_rng(6)
    n = 2000
    wi = _dirs(rng, n)
    u = rng.uniform(size=(n, 2)).astype(np.float32)
    o = _plastic_oracle()
    wo, w, pdf, typ = o.bsdf_sample(wi, u)
    spec = typ == 0x20  # EDeltaReflection
    diffuse = typ == 0x2  # EDiffuseReflection
    assert spec.any() and diffuse.any() and np.all(spec | diffuse)
    np.testing.assert_allclose(wo[spec], wi[spec] * [-1, -1, 1], atol=1e-7)  # reflect()
    # diffuse samples: weight = eval / pdf (plastic.cpp:413-416 vs :273-303)
    rgb, pdf2 = o.bsdf_eval(wi[diffuse], wo[diffuse])
    np.testing.assert_allclose(pdf[diffuse], pdf2, rtol=1e-5)
    np.testing.assert_allclose(w[diffuse], rgb / pdf2[:, None], rtol=2e-5)
    # the specular choice follows probSpecular = Fi w / (Fi w + (1 - Fi)(1 - w)) with w = 1/(1+0.9)
    sw = 1 / (1 + 0.9)
    fi = np.array([fresnel_ext(c, np.float32(1.5)) for c in wi[:, 2].astype(float)])
    ps = fi * sw / (fi * sw + (1 - fi) * (1 - sw))
    np.testing.assert_array_equal(spec, u[:, 0] < ps.astype(np.float32))


def test_twosided_flips_to_the_nested_bsdf():
    rng = np.random.default_rng(7)
    wi, wo = _dirs(rng, 300), _dirs(rng, 300)
    one = _plastic_oracle()
    two = oracle_lib.MeshOracle()
    two.new_bsdf({"type": "twosided", "nested": [{"type": "plastic", "intIOR": 1.5, "extIOR": 1.0,
                                                  "nonlinear": True, "diffuse": (0.9,) * 3, "specular": (1.0,) * 3}]})
    flip = np.array([1, 1, -1], np.float32)
    a_rgb, a_pdf = one.bsdf_eval(wi, wo)
    b_rgb, b_pdf = two.bsdf_eval(wi * flip, wo * flip)  # the back side sees the same material
    np.testing.assert_array_equal(a_rgb, b_rgb)
    np.testing.assert_array_equal(a_pdf, b_pdf)
    c_rgb, _ = two.bsdf_eval(wi, wo)
    np.testing.assert_array_equal(a_rgb, c_rgb)
    u = rng.uniform(size=(300, 2)).astype(np.float32)
    wo1, w1, p1, t1 = one.bsdf_sample(wi, u)
    wo2, w2, p2, t2 = two.bsdf_sample(wi * flip, u)
    np.testing.assert_array_equal(wo1 * flip, wo2)  # wo flipped back (twosided.cpp:172-181)
    np.testing.assert_array_equal(w1, w2)
    np.testing.assert_array_equal(p1, p2)


def test_checkerboard_texture():
    o = oracle_lib.MeshOracle()
    c0, c1 = (0.725, 0.71, 0.68), (0.325, 0.31, 0.25)
    o.new_bsdf({"type": "diffuse", "reflectanceTexture": {"type": "checkerboard", "color0": c0, "color1": c1,
                                                           "uoffset": 0.1, "voffset": -0.3, "uscale": 10,
                                                           "vscale": 7}})
    rng = np.random.default_rng(8)
    uv = rng.uniform(-0.2, 1.2, size=(500, 2)).astype(np.float32)
    wi = np.tile(np.float32([0, 0, 1]), (500, 1))
    rgb, _ = o.bsdf_eval_uv(wi, wi, uv)
    x0 = uv[:, 0] * np.float32(10) + np.float32(0.1)
    y0 = uv[:, 1] * np.float32(7) + np.float32(-0.3)
    xi = np.trunc(x0 * np.float32(2)).astype(int) % 2 * 2 - 1  # math::modulo, (int) truncates
    yi = np.trunc(y0 * np.float32(2)).astype(int) % 2 * 2 - 1
    col = np.where((xi * yi == 1)[:, None], np.float32(c0), np.float32(c1)).astype(np.float32)
    np.testing.assert_array_equal(rgb, col * np.float32(1 / np.pi))


def _mt64(o, d, v0, v1, v2):
    """float64 Moller-Trumbore: t, u (weight of v1), v (weight of v2)"""
    e1, e2 = v1 - v0, v2 - v0
    pv = np.cross(d, e2)
    det = e1 @ pv
    if abs(det) < 1e-14:
        return None
    tv = o - v0
    u = (tv @ pv) / det
    qv = np.cross(tv, e1)
    v = (d @ qv) / det
    t = (e2 @ qv) / det
    return t, u, v


def _write_obj(path, text):
    with open(path, "w") as f:
        f.write(text)
    return str(path)


def _mesh_oracle(obj=None, face_normals=False, flip_normals=False, flip_tex=True, rect=None):
    o = oracle_lib.MeshOracle()
    b = o.new_bsdf({"type": "diffuse", "diffuse": (0.5, 0.5, 0.5)})
    eye = oracle_lib.f32(np.eye(4)).reshape(16)
    if obj:
        o.check(o.lib.orc_add_obj(o.s, obj.encode(), oracle_lib.p(eye, oracle_lib._f), int(face_normals),
                                  int(flip_normals), int(flip_tex), b))
    if rect is not None:
        m = oracle_lib.f32(rect).reshape(16)
        o.check(o.lib.orc_add_rectangle(o.s, oracle_lib.p(m, oracle_lib._f), 0, b))
    return o


def test_triaccel_against_float64(tmp_path):
    rng = np.random.default_rng(9)
    V = rng.uniform(-1, 1, size=(60, 3)).astype(np.float32)
    lines = ["v %.9g %.9g %.9g" % tuple(v) for v in V] + ["f %d %d %d" % (3 * i + 1, 3 * i + 2, 3 * i + 3)
                                                         for i in range(20)]
    o = _mesh_oracle(_write_obj(tmp_path / "tri.obj", "\n".join(lines) + "\n"), face_normals=True)
    n = 4000
    org = rng.uniform(-3, 3, size=(n, 3)).astype(np.float32)
    tgt = rng.uniform(-0.8, 0.8, size=(n, 3)).astype(np.float32)
    d = tgt - org
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    t, nrm, uv, b = o.trace_scene(org, d)
    checked = 0
    for k in range(n):
        best, margin = np.inf, np.inf
        for i in range(20):
            r = _mt64(org[k].astype(float), d[k].astype(float), *V[3 * i:3 * i + 3].astype(float))
            if r is None:
                continue
            tt, u, v = r
            m = min(u, v, 1 - u - v)
            if tt > 1e-3:
                margin = min(margin, abs(m))
                if m >= 0 and tt < best:
                    best = tt
        if margin < 1e-4:
            continue  # too close to an edge for float32 to agree
        checked += 1
        if np.isinf(best):
            assert np.isinf(t[k]), k
        else:
            assert abs(t[k] - best) <= 1e-4 * max(1.0, best), (k, t[k], best)
    assert checked > 3500 and np.isfinite(t).sum() > 300


def test_obj_face_forms_and_uv_flip(tmp_path):
    # z = 0: a quad over [0, 1]^2 (a/b/c, fan of two), a triangle over [2, 3] x [0, 1] (a/b, negative
    # indices) and one (a//c) beside it -- three groups, three TriMeshes
    obj = _write_obj(tmp_path / "quad.obj", "\n".join([
        "v 0 0 0", "v 1 0 0", "v 1 1 0", "v 0 1 0", "v 2 0 0", "v 3 0 0", "v 3 1 0", "v 2 1 0",
        "vt 0 0", "vt 1 0", "vt 1 1", "vt 0 1",
        "vn 0 0 1",
        "g first", "f 1/1/1 2/2/1 3/3/1 4/4/1",
        "g second", "f -4/-4 -3/-3 -2/-2",
        "g third", "f 5//1 7//1 8//1",
    ]) + "\n")
    o = _mesh_oracle(obj)
    assert o.mesh_info() == {"meshes": 3, "triangles": 4, "vertices": 4 + 3 + 3, "rectangles": 0}
    org = np.float32([[0.25, 0.75, 1.0], [0.75, 0.25, 1.0], [2.75, 0.25, 1.0], [2.25, 0.75, 1.0]])
    d = np.float32([[0, 0, -1]] * 4)
    t, nrm, uv, b = o.trace_scene(org, d)
    np.testing.assert_allclose(t, [1] * 4, atol=1e-6)
    np.testing.assert_allclose(np.abs(nrm), [[0, 0, 1]] * 4, atol=1e-6)
    # flipTexCoords (default): v -> 1 - v (obj.cpp:303-308); the a//c mesh has no texcoords: uv = (b.y, b.z)
    np.testing.assert_allclose(uv, [[0.25, 0.25], [0.75, 0.75], [0.75, 0.75], [0.25, 0.5]], atol=1e-6)
    o2 = _mesh_oracle(obj, flip_tex=False)
    _, _, uv2, _ = o2.trace_scene(org, d)
    np.testing.assert_allclose(uv2, [[0.25, 0.75], [0.75, 0.25], [0.75, 0.25], [0.25, 0.5]], atol=1e-6)


def test_face_and_flipped_normals(tmp_path):
    # a tent of two triangles sharing the edge x = 0; no vn: smooth normals are computed
    obj = _write_obj(tmp_path / "tent.obj", "v -1 0 -1\nv 0 1 -1\nv 0 1 1\nv -1 0 1\nv 1 0 -1\nv 1 0 1\n"
                                            "f 1 2 3 4\nf 2 5 6 3\n")
    org = np.float32([[-0.5, 5, 0], [-0.01, 5, 0]])
    d = np.float32([[0, -1, 0], [0, -1, 0]])
    smooth = _mesh_oracle(obj)
    _, n_s, _, _ = smooth.trace_scene(org, d)
    face = _mesh_oracle(obj, face_normals=True)
    _, n_f, _, _ = face.trace_scene(org, d)
    s2 = np.sqrt(0.5)
    # faceNormals: the facet normal (winding (1,2,3) faces -x+y)
    np.testing.assert_allclose(np.abs(n_f[0]), [s2, s2, 0], atol=1e-6)
    # smooth: the ridge vertices average the two facets (angle-weighted, trimesh.cpp:640-672)
    assert abs(n_s[1][0]) < 0.05 and abs(n_s[1][1]) > 0.99
    flipped = _mesh_oracle(obj, flip_normals=True)
    _, n_fl, _, _ = flipped.trace_scene(org, d)
    np.testing.assert_allclose(n_fl, -n_s, atol=1e-6)


def test_rectangle(tmp_path):
    # scale x2 in x, x3 in y, then rotate +90 deg about x: the rectangle spans x in [-2, 2], z in [-3, 3] at y = 0
    m = np.array([[2, 0, 0, 0], [0, 0, -1, 0], [0, 3, 0, 0], [0, 0, 0, 1]], np.float32)
    o = _mesh_oracle(rect=m)
    org = np.float32([[1.0, 4.0, 1.5], [1.9, 4.0, -2.9], [2.1, 4.0, 0.0]])
    d = np.float32([[0, -1, 0]] * 3)
    t, nrm, uv, b = o.trace_scene(org, d)
    np.testing.assert_allclose(t[:2], [4, 4], atol=1e-6)
    assert np.isinf(t[2]) and b[2] == -1
    # normal = normalize(M^-T (0,0,1)) = -y here; uv = 0.5 (local + 1)
    np.testing.assert_allclose(nrm[:2], [[0, -1, 0]] * 2, atol=1e-6)
    np.testing.assert_allclose(uv[0], [0.5 * (0.5 + 1), 0.5 * (1.5 / 3 + 1)], atol=1e-6)


@pytest.mark.parametrize("rho", [0.25, 0.5, 0.8])
def test_integrator_diffuse_plane_under_constant_sky(rho):
    """End-to-end closed form for the C1 CPU path's integrator (path.cpp:119-294 with NEE + BSDF
    sampling under MIS, envmap sampling envmap.cpp:516-543, rectangle.cpp, diffuse.cpp): a
    diffuse plane of albedo rho that fills the view, alone under a constant unit sky, reflects
    exactly rho -- it sees nothing but the sky, so every path ends after one bounce and the
    estimator's expectation is rho * L.  The 16x16 @ 64 spp mean is within 1.5 %."""
    W = H = 16
    cam = [-1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 5, 0, 0, 0, 1]  # at z = 5, looking down -z
    js = {"sensor": {"toWorld": cam, "xfov": 30.0, "nearClip": 0.01, "farClip": 100.0},
          "integrator": {"maxDepth": 65, "rrDepth": 5, "strictNormals": True, "hideEmitters": False},
          "bsdfs": [{"type": "diffuse", "diffuse": [rho] * 3}],
          "meshes": [{"type": "rectangle", "toWorld": [4, 0, 0, 0, 0, 4, 0, 0, 0, 0, 4, 0, 0, 0, 0, 1],
                      "flipNormals": False, "bsdf": 0}],
          "emitter": {"toWorld": [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1], "scale": 1.0}}
    o = oracle_lib.MeshOracle()
    o.setup_scene(js, np.ones((16, 32, 3), np.float32), W, H, 64)
    film, _ = o.render(0, 64, threads=4, width=W, height=H)
    img = film[..., :3] / film[..., 3:4]
    assert np.all(np.isfinite(img))
    np.testing.assert_allclose(img.mean(axis=(0, 1)), [rho] * 3, rtol=0.015)
