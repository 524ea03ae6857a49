#!/usr/bin/env python3
"""C1 (BASELINE.json configs[0], the teapot plumbing scene) timed on the device and on the CPU.

The scene is tests/c1_scene.py's (models/teapot/scene.xml's structure with the stand-in meshes and
a synthetic sky).  The device renders it through the C ABI (k_mesh_paths + the film splat); the
oracle's mesh restatement renders the same scene on the host's cores (the CPU baseline, as
bench.py's cpu_baseline leg does for the hair configs).  Prints one JSON line.

  python tools/c1_timing.py [--width 64 --height 64 --spp 16 --frames 20 --cpu-threads 16]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import c1_scene  # noqa: E402
import film as ref  # noqa: E402
import oracle_lib  # noqa: E402
from mitsuba_amd import native  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--height", type=int, default=64)
    ap.add_argument("--spp", type=int, default=16)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--cpu-threads", type=int, default=16)
    a = ap.parse_args()
    d = tempfile.mkdtemp(prefix="c1_")
    xml = c1_scene.write(d)
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"w": a.width, "h": a.height, "spp": a.spp})
    t0 = time.perf_counter()
    r.prepare()
    prep_ms = (time.perf_counter() - t0) * 1e3
    r.render(0, a.spp)  # warm-up
    r.render(0, a.spp, collect_stats=True)
    s = r.stats()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        film = r.render(0, a.spp)
    gpu_ms = (time.perf_counter() - t0) * 1e3 / a.frames
    paths = a.width * a.height * a.spp
    o = oracle_lib.MeshOracle()
    o.setup_scene(r.scene_json(), ref.read_pfm(os.path.join(d, "env.pfm")), a.width, a.height, a.spp)
    t0 = time.perf_counter()
    ofilm, ostats = o.render(0, a.spp, threads=a.cpu_threads, width=a.width, height=a.height)
    cpu_ms = (time.perf_counter() - t0) * 1e3
    g, c = native.develop(film), native.develop(ofilm)
    rel = float(np.sqrt(np.mean(np.sum((g - c) ** 2, -1))) / max(float(c.mean()), 1e-12))
    print(json.dumps({
        "config": "C1 teapot structure (stand-in meshes, synthetic sky) %dx%d @ %d spp" % (a.width, a.height, a.spp),
        "paths": paths, "bounces": int(s.bounces), "prepare_ms": round(prep_ms, 2),
        "gpu_ms_per_frame": round(gpu_ms, 4), "gpu_Mpaths_s": round(paths / gpu_ms / 1e3, 2),
        "kernel_ms": {"mesh_paths": round(s.ms_shade, 4), "splat_gather": round(s.ms_gather, 4)},
        "cpu_ms_per_frame": round(cpu_ms, 2), "cpu_Mpaths_s": round(paths / cpu_ms / 1e3, 3),
        "cpu_threads": a.cpu_threads, "cpu_kind": "port (oracle mesh restatement)",
        "rel_rmse_vs_oracle": rel}))


if __name__ == "__main__":
    main()
