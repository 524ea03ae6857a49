"""Shared scene setup for parity tests: one config -> product context + oracle.

The oracle receives the scene as raw inputs (camera matrix, hair file, BSDF
parameters, environment bitmap) and re-derives everything else itself
(hair loading + merging, AABB, BSDF tables, envmap CDFs).  Only the kd-tree
node/index arrays are taken from the product's host builder; the oracle
checks them against a brute-force intersection (tests/test_host.py).
"""
from __future__ import annotations

import os
import tempfile

import numpy as np

import oracle_lib  # noqa: F401  (puts the package on sys.path)
from mitsuba_amd import native, scenes

WORK = os.environ.get("HPT_TEST_WORK", os.path.join(tempfile.gettempdir(), "hpt_test_work"))


def config_params(name):
    cfg = scenes.CONFIGS[name]
    cam = np.array([float(x) for x in cfg["cam"].split()], np.float32)
    if 'type="marschner"' in cfg["bsdf"]:
        bsdf = {"type": "marschner", "eta": np.float32(1.55) / np.float32(1.0), "distribution": "ggx",
                "alpha": 0.2, "diffuse": (0.143016, 0.0156076, 1.80928e-005), "specular": (0.5, 0.5, 0.5)}
    elif "marschnerdielectric" in cfg["bsdf"]:
        c = (0.143016, 0.0156076, 1.80928e-005)
        bsdf = {"type": "marschnerdielectric", "eta": np.float32(1.55) / np.float32(1.0), "diffuse": c,
                "specular": c, "transmittance": c}
    elif "roughplastic" in cfg["bsdf"]:
        bsdf = {"type": "roughplastic", "eta": np.float32(1.55) / np.float32(1.0), "distribution": "ggx",
                "alpha": 0.2, "sample_visible": True, "nonlinear": False,
                "diffuse": (0.143016, 0.0156076, 1.80928e-005), "specular": (1.0, 1.0, 1.0)}
    else:
        bsdf = {"type": "kajiyakay", "kd": (0.143016, 0.0156076, 1.80928e-005), "ks": (0.2, 0.2, 0.2),
                "exponent": 10.0}
    return cfg, cam, bsdf


def make(name, n_strands, width, height, spp, max_depth=None, device=native.HOST_ONLY):
    """Return (xml_path, product Renderer (prepared), Oracle (prepared, with product kd-tree))."""
    cfg, cam, bsdf = config_params(name)
    max_depth = cfg["max_depth"] if max_depth is None else max_depth
    xml = scenes.make_scene(name, WORK, n_strands=n_strands)
    r = native.Renderer(device=device)
    r.load_scene_xml(xml, {"width": width, "height": height, "spp": spp, "maxDepth": max_depth})
    r.prepare()
    env = r.envmap()
    nodes, idx, _ = r.kdtree()
    o = oracle_lib.Oracle()
    hair_file = os.path.join(WORK, "%s_%d.mitshair" % (cfg["geom"], n_strands))
    o.setup(cam, 35.0, width, height, hair_file, float(cfg["radius"]), bsdf, env, max_depth, spp=spp)
    o.set_kdtree(nodes, idx)
    o.prepare()
    return xml, r, o


def reference_flags_floor(name, n_strands, r, width, height, spp):
    """L2 between the strict oracle and the oracle built with the reference's
    own compiler flags (liboracle_ref.so): the float-nondeterminism floor that
    any re-implementation of the path inherits (SURVEY.md 7 'Hard parts' i)."""
    cfg, cam, bsdf = config_params(name)
    hair_file = os.path.join(WORK, "%s_%d.mitshair" % (cfg["geom"], n_strands))
    films = []
    nodes, idx, _ = r.kdtree()
    for variant in ("parity", "ref"):
        o = oracle_lib.Oracle(variant=variant)
        o.setup(cam, 35.0, width, height, hair_file, float(cfg["radius"]), bsdf, r.envmap(), cfg["max_depth"],
                spp=spp)
        o.set_kdtree(nodes, idx)
        o.prepare()
        films.append(native.develop(o.render(0, spp, threads=16, width=width, height=height)[0]))
    a, b = films
    same = np.all(np.abs(a - b) <= 1e-5 * np.abs(a) + 1e-7, axis=-1)
    return l2_metrics(a, b), float(same.mean())


def l2_metrics(a, b):
    """Per-pixel L2 on linear HDR RGB: RMSE of ||dRGB||, max, relative RMSE."""
    d = np.linalg.norm(a.astype(np.float64) - b.astype(np.float64), axis=-1)
    rmse = float(np.sqrt(np.mean(d * d)))
    lum = a.astype(np.float64) @ np.array([0.212671, 0.715160, 0.072169])
    return {"rmse": rmse, "max": float(d.max()), "rel_rmse": rmse / max(float(lum.mean()), 1e-12)}
