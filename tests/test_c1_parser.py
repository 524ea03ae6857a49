"""Scene-XML coverage of the C1 plugins (obj / rectangle / plastic / twosided / checkerboard):
defaults resolved as the reference's constructors do, and the reference's own errors.
Small synthetic scenes; no reference tree needed.  CPU only."""
import pytest

import oracle_lib  # noqa: F401  (puts the package on sys.path)
from mitsuba_amd import native

HEAD = '<scene version="0.6.0"><integrator type="path"/><sensor type="perspective"/>'
TAIL = '<emitter type="sunsky"><vector name="sunDirection" x="0" y="1" z="0"/></emitter></scene>'


def _load(tmp_path, body):
    p = tmp_path / "s.xml"
    p.write_text(HEAD + body + TAIL)
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(str(p))
    return r, r.scene_json()


def test_defaults(tmp_path):
    (tmp_path / "m.obj").write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    _, js = _load(tmp_path, '<shape type="obj"><string name="filename" value="m.obj"/>'
                            '<bsdf type="plastic"/></shape>'
                            '<shape type="rectangle"><boolean name="flipNormals" value="true"/>'
                            '<bsdf type="diffuse"><texture name="reflectance" type="checkerboard">'
                            '<float name="uvscale" value="4"/></texture></bsdf></shape>'
                            '<shape type="obj"><string name="filename" value="m.obj"/>'
                            '<boolean name="faceNormals" value="true"/><boolean name="flipTexCoords" value="false"/>'
                            '</shape>')
    obj, rect, obj2 = js["meshes"]
    assert obj["filename"] == str(tmp_path / "m.obj")
    assert (obj["faceNormals"], obj["flipNormals"], obj["flipTexCoords"]) == (False, False, True)
    assert (obj2["faceNormals"], obj2["flipTexCoords"]) == (True, False)
    assert rect["flipNormals"] is True and rect["toWorld"] == [1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1]
    pl = js["bsdfs"][obj["bsdf"]]
    # plastic.cpp:145-166: polypropylene / air (ior.h: 1.49 / 1.000277), specular 1, diffuse 0.5, linear
    assert pl["type"] == "plastic" and abs(pl["intIOR"] - 1.49) < 1e-6 and abs(pl["extIOR"] - 1.000277) < 1e-6
    assert pl["specular"] == [1, 1, 1] and pl["diffuse"] == [0.5, 0.5, 0.5] and pl["nonlinear"] is False
    assert pl["ensureEnergyConservation"] is True  # bsdf.cpp:30-31 default
    tex = js["bsdfs"][rect["bsdf"]]["reflectanceTexture"]
    # checkerboard.cpp:49-51 colours, texture.cpp:82-91 uvscale -> uscale / vscale
    assert tex["color0"] == pytest.approx([0.4] * 3) and tex["color1"] == pytest.approx([0.2] * 3)
    assert (tex["uscale"], tex["vscale"], tex["uoffset"], tex["voffset"]) == (4, 4, 0, 0)
    # a shape without a BSDF gets Shape::configure's 0.5 diffuse
    assert js["bsdfs"][obj2["bsdf"]]["type"] == "diffuse"


@pytest.mark.parametrize("body,msg", [
    ('<shape type="rectangle"><bsdf type="twosided"/></shape>', "nested one-sided material is required"),
    ('<shape type="rectangle"><bsdf type="twosided"><bsdf type="diffuse"/><bsdf type="diffuse"/>'
     '<bsdf type="diffuse"/></bsdf></shape>', "No more than two nested"),
    ('<shape type="rectangle"><bsdf type="twosided"><bsdf type="thindielectric"/></bsdf></shape>',
     "without a transmission component"),
    ('<shape type="rectangle"><bsdf type="plastic"><float name="intIOR" value="-1"/></bsdf></shape>', "positive"),
    ('<shape type="rectangle"><bsdf type="plastic"><texture name="diffuseReflectance" type="checkerboard"/>'
     '</bsdf></shape>', "constant colours only"),
    ('<shape type="rectangle"><bsdf type="diffuse"><texture name="reflectance" type="bitmap"/></bsdf></shape>',
     "only \"checkerboard\""),
    ('<shape type="rectangle"><bsdf type="diffuse"><texture name="reflectance" type="checkerboard">'
     '<string name="coordinates" value="xyz"/></texture></bsdf></shape>', "Only UV coordinates"),
    ('<shape type="obj"><string name="filename" value="m.obj"/><float name="maxSmoothAngle" value="30"/></shape>',
     "maxSmoothAngle"),
    ('<shape type="sphere"/>', "outside this path"),
    ('<shape type="rectangle"><bsdf type="conductor"/></shape>', "outside this path"),
])
def test_errors(tmp_path, body, msg):
    with pytest.raises(native.HairPTError, match=msg):
        _load(tmp_path, body)
