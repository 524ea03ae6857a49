#!/usr/bin/env python3
"""Per-launch kernel timeline of one frame shard (rank r of N), for the scaling analysis.

Run under rocprofv3 --kernel-trace (scripts/gpu_timeline.sh); this script only renders
(one warm-up frame, then the shard --reps times).  Summarise the database with --summarize."""
import argparse
import glob
import os
import sqlite3
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd"))


def render(a):
    import torch
    from mitsuba_amd import native, scenes
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_tl"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                           "maxDepth": cfg["max_depth"]})
    r.prepare()
    film = torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0")
    r.render_device(film.data_ptr(), 0, cfg["spp"], shard=a.shard, n_shards=a.n)
    for _ in range(a.reps):
        torch.cuda.synchronize()
        r.render_device(film.data_ptr(), 0, cfg["spp"], shard=a.shard, n_shards=a.n)
    torch.cuda.synchronize()


def summarize(path, frames):
    db = sqlite3.connect(glob.glob(os.path.join(path, "*.db"))[0])
    rows = db.execute("select k.kernel_name, d.start, d.end from kernels d join "
                      "(select id, kernel_name from rocpd_info_kernel_symbol) k on d.kernel_id = k.id "
                      "order by d.start").fetchall() if False else None
    # rocpd schema differs across versions: fall back to the 'kernels' view
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    rows = [r for r in rows if r[0].startswith("k_")]
    # the last frame: from the last k_camera on
    last = max(i for i, r in enumerate(rows) if r[0] == "k_camera")
    fr = rows[last:]
    t0 = fr[0][1]
    print("| # | kernel | start (us) | duration (us) | gap before (us) |")
    print("|---|---|---:|---:|---:|")
    prev = t0
    for i, (n, s, e) in enumerate(fr):
        print("| %d | %s | %.1f | %.1f | %.1f |" % (i, n, (s - t0) / 1e3, (e - s) / 1e3, (s - prev) / 1e3))
        prev = e
    print("\nframe span %.3f ms, kernels %.3f ms" % ((fr[-1][2] - t0) / 1e6, sum(e - s for _, s, e in fr) / 1e6))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--summarize", default=None, help="rocpd output directory to summarise instead of rendering")
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize, 1)
    else:
        render(a)
