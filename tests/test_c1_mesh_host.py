"""C1's mesh path on the host (CPU, no device): the product's own OBJ / rectangle loading, BSDF
records and BVH (csrc/host/mesh.cpp) through hpt_prepare on a host-only context, checked against
the oracle's mesh restatement (oracle/mesh_geom.h), and the scenes the mesh path refuses.
The device render of the same scene is tests/test_gpu_c1.py."""
import os

import numpy as np
import pytest

import c1_scene
import oracle_lib
from mitsuba_amd import native, synth_hair

import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import film as ref  # noqa: E402


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    d = tmp_path_factory.mktemp("c1host")
    xml = c1_scene.write(d)
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(xml, {"w": 64, "h": 64, "spp": 4})
    r.prepare()
    return {"dir": d, "r": r, "js": r.scene_json(), "env": ref.read_pfm(str(d / "env.pfm"))}


def test_mesh_scene_loads_like_the_oracle(host):
    info = host["r"].info()
    o = oracle_lib.MeshOracle()
    o.setup_scene(host["js"], host["env"], 64, 64, 4)
    mi = o.mesh_info()
    assert mi["meshes"] == 3 and mi["rectangles"] == 1
    # obj.cpp's vertex merge and fan triangulation: the same vertex and primitive counts
    assert info.vertices == mi["vertices"]
    assert info.kd_indices == mi["triangles"] + mi["rectangles"]
    # a BVH over ~11 k primitives: median splits, leaves of <= 4
    assert info.kd_nodes == 2 * ((info.kd_indices + 3) // 4) - 1 or info.kd_nodes < 2 * info.kd_indices
    assert 12 <= info.kd_depth < 64
    # the bounds enclose the floor rectangle (|x|, |z| up to 56.5) and the body (height ~6.6),
    # enlarged as gkdtree.h:1213-1220
    lo, hi = np.array(info.aabb_min), np.array(info.aabb_max)
    assert lo[0] < -56 and hi[0] > 56 and lo[2] < -56 and hi[2] > 56
    assert lo[1] < 0 < 6 < hi[1]
    np.testing.assert_array_equal(host["r"].envmap(), host["env"])


def test_host_only_context_cannot_render_mesh_scene(host):
    with pytest.raises(native.HairPTError, match="host-only"):
        host["r"].render(0, 1)


def _write_scene(d, shapes):
    body = c1_scene.SCENE
    cut = body.index("  <shape type=\"rectangle\">")
    end = body.index("  <emitter")
    return body[:cut] + shapes + body[end:]


def test_mixed_hair_and_mesh_scene_is_refused(tmp_path):
    c1_scene.write(tmp_path)
    synth_hair.write_binary_hair(str(tmp_path / "h.mitshair"),
                                 [np.array([[0, 0, 0], [0, 1, 0], [0, 2, 0.1]], np.float32)])
    shapes = ('  <shape type="hair"><string name="filename" value="h.mitshair"/><ref id="Floor"/></shape>\n'
              '  <shape type="obj"><string name="filename" value="models/Mesh000.obj"/><ref id="Material"/></shape>\n')
    (tmp_path / "mixed.xml").write_text(_write_scene(tmp_path, shapes))
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(tmp_path / "mixed.xml"))
    with pytest.raises(native.HairPTError, match="mixes hair"):
        r.prepare()


def test_mesh_path_refuses_what_it_does_not_render(tmp_path):
    c1_scene.write(tmp_path)
    # a BSDF the mesh path has no kernel for
    shapes = ('  <shape type="obj"><string name="filename" value="models/Mesh000.obj"/>\n'
              '    <bsdf type="roughplastic"/></shape>\n')
    (tmp_path / "rp.xml").write_text(_write_scene(tmp_path, shapes))
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(tmp_path / "rp.xml"))
    with pytest.raises(native.HairPTError, match="outside this path"):
        r.prepare()
    # a missing mesh file: obj.cpp's message
    shapes = '  <shape type="obj"><string name="filename" value="models/none.obj"/><ref id="Material"/></shape>\n'
    (tmp_path / "missing.xml").write_text(_write_scene(tmp_path, shapes))
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(tmp_path / "missing.xml"))
    with pytest.raises(native.HairPTError, match="not found"):
        r.prepare()


def _obj_scene(tmp_path, obj_text, name="m.obj"):
    c1_scene.write(tmp_path)
    (tmp_path / name).write_text(obj_text)
    shapes = '  <shape type="obj"><string name="filename" value="%s"/><ref id="Material"/></shape>\n' % name
    path = tmp_path / ("s_%s.xml" % name.replace(".", "_"))
    path.write_text(_write_scene(tmp_path, shapes))
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(path))
    return r


def test_obj_edge_cases(tmp_path):
    # obj.cpp:371-390 / 608-715: a quad as a fan, negative (relative) indices, `v//vn` and `v/vt`
    # faces, a degenerate triangle (TriAccel k = 3: loaded, never hit), a trailing '\' continuation
    obj = ("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvn 0 0 1\nvt 0 0\nvt 1 0\nvt 1 1\n"
           "f 1//1 2//1 3//1 4//1\n"
           "f -4/1 -3/2 \\\n -2/3\n"
           "f 1 1 2\n")
    r = _obj_scene(tmp_path, obj)
    r.prepare()
    info = r.info()
    assert info.kd_indices == 2 + 1 + 1  # the fan's two triangles, the relative-index one, the degenerate one
    o = oracle_lib.MeshOracle()
    o.setup_scene(r.scene_json(), c1_scene.synthetic_sky(), 16, 16, 1)
    assert info.vertices == o.mesh_info()["vertices"]
    # out-of-range indices and material libraries fail loudly, as obj.cpp does
    with pytest.raises(native.HairPTError, match="vertex"):
        _obj_scene(tmp_path, "v 0 0 0\nv 1 0 0\nf 1 2 7\n", "bad.obj").prepare()
    with pytest.raises(native.HairPTError, match="mtllib"):
        _obj_scene(tmp_path, "mtllib x.mtl\nv 0 0 0\n", "mtl.obj").prepare()


def test_fresnel_diffuse_reflectance_equals_the_oracle():
    """The product's adaptive Gauss-Lobatto (mesh.cpp, util.cpp:808-859 over quad.cpp:287-409) that
    configures plastic's diffuse term gives the oracle's value bit for bit (oracle/lobatto.h,
    itself within 2e-5 of scipy's float64 quadrature, tests/test_c1_mesh_pins.py)."""
    import ctypes as C
    lib = native.load_library()
    eta = np.array([1.5, 1 / 1.5, 1.33, 1 / 1.33, 1.000277, 2.4, 1.0], np.float32)
    out = np.zeros_like(eta)
    assert lib.hpt_debug_fresnel_diffuse(len(eta), eta.ctypes.data_as(C.POINTER(C.c_float)),
                                         out.ctypes.data_as(C.POINTER(C.c_float))) == 0
    ref = np.array([oracle_lib.fresnel_diffuse_reflectance(float(e)) for e in eta], np.float32)
    np.testing.assert_array_equal(out, ref)
    assert out[-1] == 0.0 and 0.05 < out[0] < 0.15  # eta = 1 reflects nothing; glass ~0.09
