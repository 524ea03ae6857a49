#!/usr/bin/env python3
"""Sweep kd-tree build parameters on the CPU: node visits / primitive tests per
ray (oracle traversal over the product's tree) for the bench scene.  The tree
never changes an image, only the traversal work; use this to choose GPU
defaults, then time the winners on the GPU with bench.py --kd ..."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import oracle_lib  # noqa: E402
import scene_util  # noqa: E402
from mitsuba_amd import native, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--strands", type=int, default=40000)
    ap.add_argument("--res", type=int, default=96)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("variants", nargs="*", help="k=v,k=v ... (kd property names)")
    a = ap.parse_args()
    cfg, cam, bsdf = scene_util.config_params(a.config)
    xml = scenes.make_scene(a.config, scene_util.WORK, n_strands=a.strands)
    hair_file = os.path.join(scene_util.WORK, "%s_%d.mitshair" % (cfg["geom"], a.strands))
    variants = a.variants or [""]
    for i, v in enumerate(variants):
        kd = dict(kv.split("=") for kv in v.split(",") if kv)
        x = scenes.with_kd_params(xml, kd, "kd%d" % i)
        r = native.Renderer(device=native.HOST_ONLY)
        r.load_scene_xml(x, {"width": a.res, "height": a.res, "spp": a.spp, "maxDepth": cfg["max_depth"]})
        t0 = time.time()
        r.prepare()
        tb = time.time() - t0
        si = r.info()
        nodes, idx, _ = r.kdtree()
        o = oracle_lib.Oracle()
        o.setup(cam, 35.0, a.res, a.res, hair_file, float(cfg["radius"]), bsdf, r.envmap(), cfg["max_depth"], spp=a.spp)
        o.set_kdtree(nodes, idx)
        o.prepare()
        _, st = o.render(0, a.spp, threads=8, width=a.res, height=a.res)
        rays = st[0] + st[1]
        print("%-60s nodes %8d leaves/idx %8d depth %2d build %.2fs | nodes/ray %.1f prims/ray %.2f"
              % (v or "reference defaults", si.kd_nodes, idx.size, si.kd_depth, tb, st[2] / rays, st[3] / rays), flush=True)


if __name__ == "__main__":
    main()
