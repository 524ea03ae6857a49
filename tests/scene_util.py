"""Shared scene setup for parity tests: one config -> product context + oracle.

The oracle receives the scene as raw inputs (camera matrix, hair file, BSDF
parameters, sunsky parameters) and re-derives everything else itself (hair
loading + merging, AABB, BSDF tables, its own sunsky bitmap, envmap CDFs).  Only the kd-tree
node/index arrays are taken from the product's host builder; the oracle
checks them against a brute-force intersection (tests/test_host.py).
"""
from __future__ import annotations

import os
import re
import tempfile

import numpy as np

import oracle_lib  # noqa: F401  (puts the package on sys.path)
from mitsuba_amd import native, scenes

WORK = os.environ.get("HPT_TEST_WORK", os.path.join(tempfile.gettempdir(), "hpt_test_work"))


def _bsdf_blocks(xml_text):
    """{id: oracle BSDF dict} from the <bsdf> blocks of a config, with each
    plugin's defaults (marschner_diffuse.cpp:113-160, kajiyakay.cpp:60-69,
    roughplastic.cpp:197-227, marschnerdielectric.cpp:147-169,
    thindielectric.cpp:73-89, diffuse.cpp:62-69)."""
    out = {}
    for m in re.finditer(r'<bsdf type="(\w+)" id="(\w+)"\s*>(.*?)</bsdf>', xml_text, re.S):
        kind, bid, body = m.groups()
        props = {}
        for k, name, val in re.findall(r'<(float|rgb|string|boolean)\s+name="(\w+)"\s+value="([^"]*)"', body):
            if k == "rgb":
                v = [float(x) for x in val.replace(",", " ").split()]
                props[name] = tuple(v * 3 if len(v) == 1 else v)
            elif k == "float":
                props[name] = float(val)
            elif k == "boolean":
                props[name] = val.lower() == "true"
            else:
                props[name] = val
        eta = np.float32(props.get("intIOR", 1.5046)) / np.float32(props.get("extIOR", 1.000277))
        if kind == "marschner":
            b = {"type": kind, "eta": eta, "distribution": props.get("distribution", "beckmann"),
                 "alpha": props.get("alpha", 0.1), "diffuse": props.get("diffuseReflectance", (0.5,) * 3),
                 "specular": props.get("specularReflectance", (0.5,) * 3)}
        elif kind == "kajiyakay":
            b = {"type": kind, "kd": props.get("diffuseReflectance", (0.5,) * 3),
                 "ks": props.get("specularReflectance", (0.2,) * 3), "exponent": props.get("exponent", 30.0)}
        elif kind == "roughplastic":
            eta = np.float32(props.get("intIOR", 1.49)) / np.float32(props.get("extIOR", 1.000277))
            b = {"type": kind, "eta": eta, "distribution": props.get("distribution", "beckmann"),
                 "alpha": props.get("alpha", 0.1), "sample_visible": props.get("sampleVisible", True),
                 "nonlinear": props.get("nonlinear", False), "diffuse": props.get("diffuseReflectance", (0.5,) * 3),
                 "specular": props.get("specularReflectance", (1.0,) * 3)}
        elif kind == "marschnerdielectric":
            eta = np.float32(props.get("intIOR", 1.501)) / np.float32(props.get("extIOR", 1.000277))
            b = {"type": kind, "eta": eta, "diffuse": props.get("diffuseReflectance", (0.5,) * 3),
                 "specular": props.get("specularReflectance", (0.1,) * 3),
                 "transmittance": props.get("specularTransmittance", (0.1,) * 3)}
        elif kind == "thindielectric":
            b = {"type": kind, "eta": eta, "specular": props.get("specularReflectance", (1.0,) * 3),
                 "transmittance": props.get("specularTransmittance", (1.0,) * 3)}
        else:
            b = {"type": "diffuse", "diffuse": props.get("reflectance", props.get("diffuseReflectance", (0.5,) * 3))}
        out[bid] = b
    return out


def config_params(name):
    """(config, camera matrix, BSDF of the first shape) -- single-shape callers."""
    cfg = scenes.CONFIGS[name]
    cam = np.array([float(x) for x in cfg["cam"].split()], np.float32)
    blocks = _bsdf_blocks(cfg["bsdf"])
    return cfg, cam, blocks[cfg.get("shapes", ["hair"])[0]]


def oracle_envmap(name, resolution=512):
    """The oracle's OWN sunsky bitmap for a config (oracle/sunsky_ref.cpp, written from the
    reference; tests/test_independent_pins.py checks it bitwise against the product's and
    against a float64 restatement) -- the oracle is never lit by the product's bitmap."""
    cfg = scenes.CONFIGS[name]
    ss = scenes.SUNSKY
    return oracle_lib.sunsky_bitmap([float(x) for x in cfg["sun"].split()], float(ss["turbidity"]), 0.2, 1.0,
                                    float(ss["skyScale"]), float(ss["sunScale"]), float(ss["sunRadiusScale"]),
                                    resolution)


def oracle_shapes(name, n_strands, workdir=None, radii=None):
    """[(hair file, radius, oracle BSDF dict)] per hair shape of a config."""
    cfg = scenes.CONFIGS[name]
    files = scenes.hair_files(name, workdir or WORK, n_strands)
    blocks = _bsdf_blocks(cfg["bsdf"])
    radii = radii or [cfg["radius"]] * len(files)
    return [(f, float(rad), blocks[ref]) for f, ref, rad in zip(files, cfg.get("shapes", ["hair"]), radii)]


def make(name, n_strands, width, height, spp, max_depth=None, device=native.HOST_ONLY, radii=None, workdir=None):
    """Return (xml_path, product Renderer (prepared), Oracle (prepared, with product kd-tree))."""
    cfg, cam, _ = config_params(name)
    max_depth = cfg["max_depth"] if max_depth is None else max_depth
    xml = scenes.make_scene(name, workdir or WORK, n_strands=n_strands, **({"radii": radii} if radii else {}))
    r = native.Renderer(device=device)
    r.load_scene_xml(xml, {"width": width, "height": height, "spp": spp, "maxDepth": max_depth})
    r.prepare()
    env = oracle_envmap(name)
    nodes, idx, _ = r.kdtree()
    o = oracle_lib.Oracle()
    o.setup(cam, 35.0, width, height, oracle_shapes(name, n_strands, workdir, radii=radii), None, None, env,
            max_depth, spp=spp)
    o.set_kdtree(nodes, idx)
    o.prepare()
    return xml, r, o


def reference_flags_floor(name, n_strands, r, width, height, spp, radii=None, max_depth=None, shard=0, n_shards=1,
                          workdir=None):
    """L2 between the strict oracle and the oracle built with the reference's
    own compiler flags (liboracle_ref.so): the float-nondeterminism floor that
    any re-implementation of the path inherits (SURVEY.md 7 'Hard parts' i)."""
    cfg, cam, _ = config_params(name)
    shapes = oracle_shapes(name, n_strands, workdir, radii=radii)
    films = []
    nodes, idx, _ = r.kdtree()
    for variant in ("parity", "ref"):
        o = oracle_lib.Oracle(variant=variant)
        o.setup(cam, 35.0, width, height, shapes, None, None, oracle_envmap(name),
                cfg["max_depth"] if max_depth is None else max_depth, spp=spp)
        o.set_kdtree(nodes, idx)
        o.prepare()
        films.append(o.render(0, spp, threads=16, shard=shard, n_shards=n_shards, width=width, height=height)[0])
    mask = films[0][..., 3] > 0  # a shard's pixels (every pixel of a full frame)
    a, b = [native.develop(f)[mask] for f in films]
    same = np.all(np.abs(a - b) <= 1e-5 * np.abs(a) + 1e-7, axis=-1)
    return l2_metrics(a, b), float(same.mean())


def l2_metrics(a, b):
    """Per-pixel L2 on linear HDR RGB: RMSE of ||dRGB||, its max and 99th
    percentile over pixels, relative RMSE, and the fraction of pixels whose L2 exceeds
    north_star's 1e-3."""
    d = np.linalg.norm(a.astype(np.float64) - b.astype(np.float64), axis=-1)
    rmse = float(np.sqrt(np.mean(d * d)))
    lum = a.astype(np.float64) @ np.array([0.212671, 0.715160, 0.072169])
    return {"rmse": rmse, "max": float(d.max()), "p99": float(np.percentile(d, 99)),
            "rel_rmse": rmse / max(float(lum.mean()), 1e-12), "frac_gt_1e-3": float(np.mean(d > 1e-3))}


def assert_at_floor(m, floor, same, floor_same, factor=2.0):
    """The film-parity bar of every render test, per-pixel statistics against the same
    statistics of the reference-flags noise floor (the strict oracle vs the oracle built
    with the reference's own compiler flags):
      - RMSE below north_star's 1e-3 and within `factor` of the floor's;
      - the per-pixel maximum within `factor` of the floor's maximum (a single path that
        flips a discrete event moves its pixel by O(radiance / spp), on either side);
      - the fraction of pixels with L2 > 1e-3 at most `factor` x the floor's, + 0.2 %;
      - bit-identical pixels no fewer than the floor's, - 5 %."""
    assert m["rmse"] < 1e-3, m
    assert m["rmse"] <= factor * floor["rmse"] + 1e-6, (m, floor)
    assert m["max"] <= factor * floor["max"] + 1e-5, (m, floor)
    assert m["frac_gt_1e-3"] <= factor * floor["frac_gt_1e-3"] + 2e-3, (m, floor)
    assert same >= floor_same - 0.05, (same, floor_same)


def fold_workdir(n_strands, folded=True):
    """A work directory whose furball hair file (the name scenes.hair_files looks for) has three
    strands folded back on themselves near the camera -- an exact hairpin (a vertex returns to the
    one before last: opposite tangents, NaN miter normals, a segment no exact test accepts,
    hair.cpp:521-531), a near-exact fold (one ulp off the hairpin: a miter plane almost parallel to
    the axis, so the segment's axial reach is ~1e5 radii) and a 179.9 degree fold -- or, with
    folded=False, the same furball unfolded (the fold-free twin).  Scenes made with
    scenes.make_scene(..., workdir) / make(..., workdir=) read it."""
    d = os.path.join(WORK, "folds_%d_%d" % (n_strands, int(folded)))
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "furball_%d.mitshair" % n_strands)
    if os.path.exists(path):
        return d
    strands = [np.asarray(x, np.float32).copy() for x in scenes.synth_hair.furball(n_strands)]
    if folded:
        cam = np.array([float(x) for x in scenes.FURBALL_CAM.split()]).reshape(4, 4)[:3, 3]
        near = np.argsort([np.linalg.norm(x[0] - cam) for x in strands])
        pick = [int(k) for k in near if len(strands[k]) >= 6][:3]
        hp, nf, f179 = (strands[k] for k in pick)
        hp[3] = hp[1]                                          # exact hairpin at vertex 2
        nf[3] = nf[1]
        nf[3, 0] = np.nextafter(nf[3, 0], np.float32(np.inf))  # one ulp off it
        back = (f179[1] - f179[2]).astype(np.float64)          # 179.9 degrees at vertex 2
        side = np.cross(back, [0.3, 1.0, 0.2])
        side /= np.linalg.norm(side)
        ang = np.radians(0.1)
        f179[3] = (f179[2] + np.cos(ang) * back + np.sin(ang) * np.linalg.norm(back) * side).astype(np.float32)
    tmp = path + ".tmp%d" % os.getpid()
    scenes.synth_hair.write_binary_hair(tmp, strands)
    os.replace(tmp, path)
    return d
