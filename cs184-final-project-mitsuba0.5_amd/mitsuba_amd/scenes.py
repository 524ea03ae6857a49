"""Benchmark / parity scene configurations (BASELINE.json "configs").

Each config is a Mitsuba scene XML mirroring the reference's models/ scenes
(camera matrices, fov, hair radius, BSDF and sunsky parameters copied as
numbers from models/*/scene*.xml) with synthetic hair written next to it:

  straight_kk      models/straight-hair/scene_kkay.xml       kajiyakay  256^2 @ 64
  furball_marschner models/furball/scene.xml + the marschner block of
                   models/straight-hair/scene_marschner.xml:31-39   512^2 @ 256 (headline)
  curly_marschner  models/curly-hair/scene.xml + marschner     1024^2 @ 256
  furball_roughplastic models/furball/scene.xml as shipped (roughplastic) 512^2 @ 256
  straight_dielectric models/straight-hair/scene_dielectric.xml (marschnerdielectric) 1024^2 @ 128
  haircurl_roughplastic / haircurl_kk  models/hair-curl/{scene,kkay_scene}.xml: four hair
                   shapes with one BSDF each, 1200x1000 @ 64
  furball_1m       furball scaled to ~1M segments              1024^2 @ 1024, maxDepth 64
Resolution / spp / maxDepth are $-parameters (-D width=..., spp=...).
"""
from __future__ import annotations

import os

from . import synth_hair

FURBALL_CAM = ("-0.704024 0.0939171 0.703939 -10.6677 1.05829e-008 0.991217 -0.132245 14.3141 "
               "-0.710177 -0.0931033 -0.69784 10.2879 0 0 0 1")          # models/furball/scene.xml:12
STRAIGHT_CAM = ("0.999887 0.00390257 0.0145262 -0.234672 6.98571e-010 0.965755 -0.259457 16.5124 "
                "-0.0150413 0.259428 0.965645 -25.3482 0 0 0 1")          # models/straight-hair/scene*.xml:12
HAIR_DIFFUSE = "0.143016, 0.0156076, 1.80928e-005"

MARSCHNER = """  <bsdf type="marschner" id="hair">
    <float name="alpha" value="0.2"/>
    <string name="distribution" value="ggx"/>
    <float name="intIOR" value="1.55"/>
    <float name="extIOR" value="1"/>
    <boolean name="nonlinear" value="false"/>
    <rgb name="diffuseReflectance" value="%s"/>
    <float name="exponent" value="10.0"/>
  </bsdf>""" % HAIR_DIFFUSE

KAJIYAKAY = """  <bsdf type="kajiyakay" id="hair">
    <rgb name="diffuseReflectance" value="%s"/>
    <float name="exponent" value="10"/>
  </bsdf>""" % HAIR_DIFFUSE

ROUGHPLASTIC = """  <bsdf type="roughplastic" id="hair">
    <float name="alpha" value="0.2"/>
    <string name="distribution" value="ggx"/>
    <float name="intIOR" value="1.55"/>
    <float name="extIOR" value="1"/>
    <boolean name="nonlinear" value="false"/>
    <rgb name="diffuseReflectance" value="%s"/>
  </bsdf>""" % HAIR_DIFFUSE                                           # models/furball/scene.xml:31-38

MARSCHNER_DIELECTRIC = """  <bsdf type="marschnerdielectric" id="hair">
    <float name="intIOR" value="1.55"/>
    <float name="extIOR" value="1"/>
    <float name="exponent" value="5.0"/>
    <rgb name="specularTransmittance" value="%s"/>
    <rgb name="specularReflectance" value="%s"/>
    <rgb name="diffuseReflectance" value="%s"/>
  </bsdf>""" % (HAIR_DIFFUSE, HAIR_DIFFUSE, HAIR_DIFFUSE)          # models/straight-hair/scene_dielectric.xml:31-38

THIN_DIELECTRIC = """  <bsdf type="thindielectric" id="hair">
    <float name="intIOR" value="1.55"/>
    <float name="extIOR" value="1"/>
    <float name="exponent" value="5.0"/>
    <rgb name="specularTransmittance" value="%s"/>
    <rgb name="specularReflectance" value="%s"/>
  </bsdf>""" % (HAIR_DIFFUSE, HAIR_DIFFUSE)                        # models/straight-hair/scene_thindielectric.xml:31-37

# thindielectric with unit weights: every bounce keeps throughput 1, so only Russian
# roulette (q = 0.95) ends a path -- the long-path case of maxDepth = -1 (tests)
THIN_DIELECTRIC_WHITE = THIN_DIELECTRIC.replace(HAIR_DIFFUSE, "1, 1, 1")

HAIRCURL_CAM = ("-1 4.24672e-010 1.50958e-007 -0.055286 1.11022e-016 0.999996 -0.00281317 5.92976 "
                "-1.50959e-007 -0.00281317 -0.999996 17.0651 0 0 0 1")      # models/hair-curl/scene.xml:12
HAIRCURL_COLOURS = [("black_hair", "6.344e-006, 7.62186e-012, 6.53751e-030"),
                    ("red_hair", "0.0112431, 6.77287e-005, 1.13705e-011"),
                    ("brown_hair", "0.143016, 0.0156076, 1.80928e-005"),
                    ("blonde_hair", "0.592384, 0.32628, 0.0528657")]      # models/hair-curl/*.xml:31-65
HAIRCURL_RP = "\n".join("""  <bsdf type="roughplastic" id="%s">
    <float name="alpha" value="0.3"/>
    <string name="distribution" value="ggx"/>
    <float name="intIOR" value="1.55"/>
    <float name="extIOR" value="1"/>
    <boolean name="nonlinear" value="false"/>
    <rgb name="diffuseReflectance" value="%s"/>
  </bsdf>""" % c for c in HAIRCURL_COLOURS)                           # models/hair-curl/scene.xml
HAIRCURL_KK = "\n".join("""  <bsdf type="kajiyakay" id="%s">
    <float name="exponent" value="10"/>
    <rgb name="diffuseReflectance" value="%s"/>
  </bsdf>""" % c for c in HAIRCURL_COLOURS)                           # models/hair-curl/kkay_scene.xml

CONFIGS = {
    # name: (camera, bsdf, radius, sun direction, width, height, spp, maxDepth, geometry, geometry args)
    "straight_kk": dict(cam=STRAIGHT_CAM, bsdf=KAJIYAKAY, radius="0.00566563", sun="0.19033 0.758426 -0.623349",
                        width=256, height=256, spp=64, max_depth=65, geom="straight", n=10000),
    "furball_marschner": dict(cam=FURBALL_CAM, bsdf=MARSCHNER, radius="0.00216667", sun="-0.376047 0.758426 0.532333",
                              width=512, height=512, spp=256, max_depth=65, geom="furball", n=40000),
    "curly_marschner": dict(cam=STRAIGHT_CAM, bsdf=MARSCHNER, radius="0.00559955", sun="0.19033 0.758426 -0.623349",
                            width=1024, height=1024, spp=256, max_depth=65, geom="curly", n=10000),
    "furball_roughplastic": dict(cam=FURBALL_CAM, bsdf=ROUGHPLASTIC, radius="0.00216667",
                                 sun="-0.376047 0.758426 0.532333", width=512, height=512, spp=256, max_depth=65,
                                 geom="furball", n=40000),
    "straight_dielectric": dict(cam=STRAIGHT_CAM, bsdf=MARSCHNER_DIELECTRIC, radius="0.00566563",
                                sun="0.19033 0.758426 -0.623349", width=1024, height=1024, spp=128, max_depth=65,
                                geom="straight", n=10000),
    # four hair shapes, one BSDF each (models/hair-curl: 1200x1000 @ 64 spp, radius 0.000444)
    "haircurl_roughplastic": dict(cam=HAIRCURL_CAM, bsdf=HAIRCURL_RP, radius="0.000444",
                                  sun="-0.376047 0.758426 0.532333", width=1200, height=1000, spp=64, max_depth=65,
                                  geom="curl4", n=6000, shapes=[c[0] for c in HAIRCURL_COLOURS]),
    "haircurl_kk": dict(cam=HAIRCURL_CAM, bsdf=HAIRCURL_KK, radius="0.000444", sun="-0.376047 0.758426 0.532333",
                        width=1200, height=1000, spp=64, max_depth=65, geom="curl4", n=6000,
                        shapes=[c[0] for c in HAIRCURL_COLOURS]),
    "straight_thindielectric": dict(cam=STRAIGHT_CAM, bsdf=THIN_DIELECTRIC, radius="0.00566563",
                                    sun="0.19033 0.758426 -0.623349", width=1024, height=1024, spp=128, max_depth=65,
                                    geom="straight", n=10000),
    "furball_thin_white": dict(cam=FURBALL_CAM, bsdf=THIN_DIELECTRIC_WHITE, radius="0.00216667",
                               sun="-0.376047 0.758426 0.532333", width=128, height=128, spp=16, max_depth=-1,
                               geom="furball", n=40000),
    "furball_1m": dict(cam=FURBALL_CAM, bsdf=MARSCHNER, radius="0.00216667", sun="-0.376047 0.758426 0.532333",
                       width=1024, height=1024, spp=1024, max_depth=64, geom="furball", n=125000),
}

XML = """<?xml version="1.0" encoding="utf-8"?>
<!-- generated by mitsuba_amd.scenes: {name} -->
<scene version="0.6.0">
  <default name="spp" value="{spp}"/>
  <default name="width" value="{width}"/>
  <default name="height" value="{height}"/>
  <default name="maxDepth" value="{max_depth}"/>
{hairdefaults}  <integrator type="path">
    <integer name="maxDepth" value="$maxDepth"/>
    <boolean name="strictNormals" value="true"/>
  </integrator>
  <sensor type="perspective">
    <float name="fov" value="35"/>
    <transform name="toWorld">
      <matrix value="{cam}"/>
    </transform>
    <sampler type="sobol">
      <integer name="sampleCount" value="$spp"/>
    </sampler>
    <film type="ldrfilm">
      <integer name="width" value="$width"/>
      <integer name="height" value="$height"/>
      <string name="fileFormat" value="png"/>
      <string name="pixelFormat" value="rgb"/>
      <float name="gamma" value="2.2"/>
      <boolean name="banner" value="false"/>
      <rfilter type="tent"/>
    </film>
  </sensor>
{bsdf}
{shapes}
  <emitter type="sunsky">
    <float name="turbidity" value="{turbidity}"/>
    <vector name="sunDirection" x="{sx}" y="{sy}" z="{sz}"/>
    <float name="skyScale" value="{skyScale}"/>
    <float name="sunScale" value="{sunScale}"/>
    <float name="sunRadiusScale" value="{sunRadiusScale}"/>
  </emitter>
</scene>
"""


# the sunsky block of models/furball/scene.xml and models/*-hair/scene*.xml (turbidity 3,
# skyScale 5, sunScale 19.0912, sunRadiusScale 37.9165; default resolution 512, albedo 0.2)
SUNSKY = dict(turbidity="3", skyScale="5", sunScale="19.0912", sunRadiusScale="37.9165")


def hair_strands(geom: str, n: int):
    if geom == "furball":
        return synth_hair.furball(n)
    if geom == "straight":
        return synth_hair.straight(n)
    if geom == "curly":
        return synth_hair.curly(n)
    raise ValueError(geom)


SHAPE = """  <shape type="hair">
    <float name="radius" value="{radius}"/>
    <string name="filename" value="${var}"/>
    <ref id="{ref}"/>
  </shape>"""


def hair_files(name: str, workdir: str, n_strands: int | None = None):
    """Hair file path(s) of a config (one per hair shape), written if missing."""
    cfg = CONFIGS[name]
    n = int(n_strands if n_strands is not None else cfg["n"])
    os.makedirs(workdir, exist_ok=True)
    if cfg["geom"] == "curl4":
        items = [("curl4_%d_%d.mitshair" % (k, n), lambda k=k: synth_hair.curl_lock(n, k)) for k in range(4)]
    else:
        items = [("%s_%d.mitshair" % (cfg["geom"], n), lambda: hair_strands(cfg["geom"], n))]
    out = []
    for fname, gen in items:
        path = os.path.join(workdir, fname)
        if not os.path.exists(path):
            tmp = path + ".tmp%d" % os.getpid()
            synth_hair.write_binary_hair(tmp, gen())
            os.replace(tmp, path)
        out.append(path)
    return out


def make_scene(name: str, workdir: str, n_strands: int | None = None, **override) -> str:
    """Write <workdir>/<name>_<n>.xml (+ hair files, cached) and return the XML path."""
    cfg = dict(CONFIGS[name])
    cfg.update(override)
    n = int(n_strands if n_strands is not None else cfg["n"])
    files = hair_files(name, workdir, n)
    refs = cfg.get("shapes", ["hair"])
    var = ["hairfile"] if len(files) == 1 else ["hairfile%d" % k for k in range(len(files))]
    defaults = "".join('  <default name="%s" value="%s"/>\n' % (v, os.path.basename(f)) for v, f in zip(var, files))
    radii = cfg.get("radii") or [cfg["radius"]] * len(files)   # per-shape radii (tests)
    shapes = "\n".join(SHAPE.format(radius=rad, var=v, ref=r) for v, r, rad in zip(var, refs, radii))
    sx, sy, sz = cfg["sun"].split()
    xml = XML.format(name=name, spp=cfg["spp"], width=cfg["width"], height=cfg["height"],
                     max_depth=cfg["max_depth"], hairdefaults=defaults, cam=cfg["cam"],
                     bsdf=cfg["bsdf"], shapes=shapes, sx=sx, sy=sy, sz=sz, **SUNSKY)
    path = os.path.join(workdir, "%s_%d.xml" % (name, n))
    _write_atomic(path, xml)
    return path


def _write_atomic(path: str, text: str) -> None:
    """Write via a per-process temporary + rename: ranks that write the same
    scene file concurrently never read a half-written one."""
    tmp = path + ".tmp%d" % os.getpid()
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, path)


_KD_INT = ("kdStopPrims", "kdMaxDepth", "kdMaxBadRefines", "kdClipMinPrims", "kdExactSweepMax")


def with_kd_params(xml: str, kd: dict, tag: str = "kd") -> str:
    """Copy of scene `xml` whose hair shape carries kd-tree build properties
    (kdIntersectionCost, kdTraversalCost, kdEmptySpaceBonus, kdStopPrims,
    kdMaxDepth, kdMaxBadRefines, kdClip; names of scene.cpp:44-78)."""
    import re

    props = "".join('<%s name="%s" value="%s"/>' % ("integer" if k in _KD_INT else
                                                    ("boolean" if k == "kdClip" else "float"), k, v)
                    for k, v in kd.items())
    s = open(xml).read()
    s = re.sub(r'(<shape type="hair"[^>]*>)', lambda m: m.group(1) + props, s, count=1)
    out = xml[:-4] + "_%s.xml" % tag
    _write_atomic(out, s)
    return out
