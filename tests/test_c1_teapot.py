"""C1 -- the "teapot" CPU plumbing configuration (BASELINE.json configs[0]).

models/teapot/scene.xml:31-84 (path tracer, maxDepth 65, strictNormals; two
`twosided` materials -- `plastic` and a `checkerboard` `diffuse`; a `rectangle`
floor; two `obj` meshes; an RGBE `envmap`) is loaded through the product's
C ABI (hpt_load_scene_xml, host-only context) and exported as JSON
(hpt_export_scene_json); the CPU path (the oracle's restatement of obj.cpp /
trimesh.cpp / TriAccel / rectangle.cpp / plastic.cpp / twosided.cpp /
checkerboard.cpp, oracle/mesh_*.h) renders it at 64 x 64 @ 16 spp.  The product
prepares the same scene with its own loader (csrc/host/mesh.cpp); its device render
(k_mesh_paths) is checked against the oracle in tests/test_gpu_c1.py.

The reference does not ship models/Mesh00{0,1}.obj: tests/teapot_meshes.py
writes seeded stand-ins.  The scene file and its envmap are read from
/root/reference at test time (this file is CPU-only; the GPU box has no
reference tree); no pixel of a reference render exists for these meshes, so
the render is checked for determinism and by geometric probes -- parity of the
mesh path against the reference is unpinned beyond the unit pins below.
"""
import os
import shutil
import struct
import sys
import zlib

import numpy as np
import pytest

import oracle_lib
import teapot_meshes
from mitsuba_amd import native

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import film as ref  # noqa: E402

REF_TEAPOT = "/root/reference/models/teapot"
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF_TEAPOT, "scene.xml")),
                                reason="the reference's teapot scene is only present in the build container")

W = H = 64
SPP = 16


@pytest.fixture(scope="module")
def teapot(tmp_path_factory):
    d = tmp_path_factory.mktemp("teapot")
    shutil.copy(os.path.join(REF_TEAPOT, "scene.xml"), d / "scene.xml")
    os.symlink(os.path.join(REF_TEAPOT, "textures"), d / "textures")
    teapot_meshes.write_all(str(d / "models"))
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(d / "scene.xml"))
    js = r.scene_json()
    env, _ = ref.read_rgbe(os.path.join(REF_TEAPOT, "textures", "envmap.hdr"))
    o = oracle_lib.MeshOracle()
    table = o.setup_scene(js, env, W, H, SPP)
    return {"dir": d, "r": r, "js": js, "o": o, "table": table}


def test_scene_parses_through_the_c_abi(teapot):
    js, d = teapot["js"], teapot["dir"]
    it, sen = js["integrator"], js["sensor"]
    assert (it["type"], it["maxDepth"], it["rrDepth"], it["strictNormals"], it["hideEmitters"]) == \
        ("path", 65, 5, True, False)
    assert (sen["fov"], sen["fovAxis"], sen["width"], sen["height"], sen["sampleCount"]) == (35, "x", 1280, 720, 64)
    assert (sen["film"], sen["rfilter"]) == ("ldrfilm", "tent")
    np.testing.assert_allclose(sen["toWorld"][:4], [-0.00550949, -0.342144, -0.939631, 23.895], rtol=1e-6)
    # two referenced materials, each a twosided wrapper (scene.xml:31-50), in first-reference order
    floor, mat = js["bsdfs"]
    assert mat["type"] == "twosided" and [n["type"] for n in mat["nested"]] == ["plastic"]
    pl = mat["nested"][0]
    assert (pl["intIOR"], pl["extIOR"], pl["nonlinear"]) == (1.5, 1.0, True)
    np.testing.assert_allclose(pl["diffuse"], [0.9] * 3, rtol=1e-6)
    np.testing.assert_allclose(pl["specular"], [1.0] * 3)
    assert floor["type"] == "twosided" and floor["nested"][0]["type"] == "diffuse"
    tex = floor["nested"][0]["reflectanceTexture"]
    assert tex["type"] == "checkerboard"
    np.testing.assert_allclose(tex["color0"], [0.725, 0.71, 0.68], rtol=1e-6)
    np.testing.assert_allclose(tex["color1"], [0.325, 0.31, 0.25], rtol=1e-6)
    assert (tex["uoffset"], tex["voffset"], tex["uscale"], tex["vscale"]) == (0, 0, 10, 10)
    # shapes in document order, BSDFs by reference
    assert [m["type"] for m in js["meshes"]] == ["rectangle", "obj", "obj"]
    assert [m["bsdf"] for m in js["meshes"]] == [0, 1, 1]
    assert js["meshes"][1]["filename"] == str(d / "models" / "Mesh001.obj")
    assert js["meshes"][2]["filename"] == str(d / "models" / "Mesh000.obj")
    assert all(m["flipTexCoords"] and not m["faceNormals"] for m in js["meshes"][1:])
    assert js["hair"] == []
    em = js["emitter"]
    assert em["type"] == "envmap" and em["filename"].endswith("textures/envmap.hdr")
    np.testing.assert_allclose(em["toWorld"][:4], [-0.922278, 0, 0.386527, 0], rtol=1e-6)


def test_product_prepares_the_teapot_like_the_oracle(teapot):
    # the product's own loader (csrc/host/mesh.cpp) behind hpt_prepare: the device path renders the
    # scene (k_mesh_paths; tests/test_gpu_c1.py checks that render against the oracle)
    r = teapot["r"]
    r.prepare()
    info, mi = r.info(), teapot["o"].mesh_info()
    assert info.vertices == mi["vertices"]
    assert info.kd_indices == mi["triangles"] + mi["rectangles"]
    with pytest.raises(native.HairPTError, match="host-only"):
        r.render(0, 1)


def test_substitute_meshes_load(teapot):
    info = teapot["o"].mesh_info()
    # Mesh001: 96x46 quads (fan -> 2 triangles) + 2x96 pole triangles, v/vt/vn all equal -> 96*47+2 vertices;
    # Mesh000: groups handle (48x16 quads, 768 vertices) and knob (24x10x2 + 48 triangles, 24*11+2 vertices)
    assert info == {"meshes": 3, "triangles": 9024 + 1536 + 528, "vertices": 4514 + 768 + 266, "rectangles": 1}


def _camera_rays(o, px, py):
    pos = np.stack([px + 0.5, py + 0.5], axis=-1).astype(np.float32)
    org, d, _, _ = o.camera_rays(pos)
    return org, d


def test_geometric_probes(teapot):
    o, table = teapot["o"], teapot["table"]
    # the pixel centre looks at the body (Material); the bottom row at the floor (Floor)
    org, d = _camera_rays(o, np.array([32.0, 32.0, 2.0, 61.0]), np.array([32.0, 24.0, 62.0, 62.0]))
    t, n, uv, b = o.trace_scene(org, d)
    floor_idx, mat_idx = table[0], table[1]
    assert b[0] == mat_idx and b[1] == mat_idx
    assert b[2] == floor_idx and b[3] == floor_idx
    assert np.all(np.isfinite(t))
    # floor uv = 0.5 (local + 1) within [0, 1]; the hit lies in y = 0 (rectangle.cpp:125-168)
    assert np.all((uv[2:] >= 0) & (uv[2:] <= 1))
    p = org[2:] + t[2:, None] * d[2:]
    assert np.all(np.abs(p[:, 1]) < 1e-3)
    # a ray straight down beside the knob hits the body sphere (centre (0, R, 0), R = 3.3, bumps 1 %)
    R, x, z = 3.3, 1.5, 0.5
    y = R + np.sqrt(R * R - x * x - z * z)
    t2, n2, _, b2 = o.trace_scene([[x, 20.0, z]], [[0.0, -1.0, 0.0]])
    assert b2[0] == mat_idx and abs((20.0 - t2[0]) - y) < 0.05
    np.testing.assert_allclose(n2[0], np.array([x, y - R, z]) / R, atol=0.02)  # interpolated vn


@pytest.fixture(scope="module")
def render(teapot):
    film, stats = teapot["o"].render(0, SPP, threads=8, width=W, height=H)
    return film, stats


def test_render_is_deterministic_and_sane(teapot, render):
    film, stats = render
    film2, stats2 = teapot["o"].render(0, SPP, threads=3, width=W, height=H)
    np.testing.assert_array_equal(film, film2)  # thread count does not change a bit
    np.testing.assert_array_equal(stats, stats2)
    img = native.develop(film)
    assert np.all(np.isfinite(img)) and np.all(img >= 0)
    assert stats[4] == W * H * SPP and stats[7] == 0  # every path, no rejected sample
    assert img.mean() > 0.05
    # the checkerboard shows on the floor: the bottom rows alternate between two albedos
    row = img[-3].mean(axis=-1)
    assert row.max() > 1.5 * row.min()


def test_render_writes_png(teapot, render, tmp_path):
    film, _ = render
    r = teapot["r"]
    params = r.film_params()
    assert (params.ldr, params.file_format, params.banner) == (1, native.FILE_PNG, 0)
    assert abs(params.gamma - 2.2) < 1e-6
    out = r.write_film(tmp_path / "teapot", film, params)
    assert out.endswith("teapot.png")
    data = open(out, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    w, h = struct.unpack(">II", data[16:24])
    assert (w, h) == (W, H)
    px = ref.read_png(out)
    np.testing.assert_array_equal(px, ref.develop_ldr(film, gamma=2.2))
    assert zlib.crc32(data) == zlib.crc32(open(r.write_film(tmp_path / "again", film, params), "rb").read())
