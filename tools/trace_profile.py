#!/usr/bin/env python3
"""Where does a k_trace launch's time go at small shards?  Renders rank r of N with a library
built with -DHPT_TRACE_PROFILE (make variant V=traceprof KFLAGS=-DHPT_TRACE_PROFILE, selected
with HAIRPT_LIB) and summarises, per k_trace launch, the per-wave records: the launch's span,
when the work queue ran dry (the first wave that found every shard empty), the drain after it
(last wave exit), how many rays were still in flight then, and the throughput before / after.

Usage: HAIRPT_LIB=.../libv_traceprof/libhairpt.so python tools/trace_profile.py [--shards 8]
"""
import argparse
import ctypes as C
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd"))

import torch  # noqa: E402

from mitsuba_amd import native, scenes  # noqa: E402

WAVES, LAUNCHES = 16384, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_traceprof"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                           "maxDepth": cfg["max_depth"]})
    r.prepare()
    lib = native.load_library()
    lib.hpt_debug_traceprof.restype = C.c_int
    lib.hpt_debug_traceprof.argtypes = [C.c_void_p, C.c_int]
    buf = np.zeros((LAUNCHES, WAVES, 8), dtype=np.uint64)
    film = torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0")
    out = []
    for rep in range(2):
        lib.hpt_debug_traceprof(buf.ctypes.data, LAUNCHES)  # clear
        film.zero_()
        r.render_device(film.data_ptr(), 0, cfg["spp"], shard=a.shard, n_shards=a.shards, collect_stats=1)
        torch.cuda.synchronize()
        got = lib.hpt_debug_traceprof(buf.ctypes.data, LAUNCHES)
        out = []
        for li in range(got):
            rec = buf[li]
            rec = rec[rec[:, 2] > 0].astype(np.float64)
            beg, ex, end, claimed, infl = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3], rec[:, 4]
            drounds, dlanes = rec[:, 5], rec[:, 6]
            t0 = beg.min()
            tdry = ex[ex > 0].min() if (ex > 0).any() else end.max()
            tick = 0.01  # us per tick (100 MHz)
            span = (end.max() - t0) * tick
            main_us = (tdry - t0) * tick
            drain = (end.max() - tdry) * tick
            ends = np.sort((end - t0) * tick)
            out.append({"launch": li, "waves": int(rec.shape[0]), "rays": int(claimed.sum()),
                        "span_us": round(span, 1), "dry_at_us": round(main_us, 1), "drain_us": round(drain, 1),
                        "start_spread_us": round((np.percentile(beg, 99) - t0) * tick, 1),
                        "in_flight_at_dry": int(infl.sum()),
                        "rays_per_us_main": round(claimed.sum() / max(main_us, 1e-9), 1),
                        "wave_end_pct_us": {p: round(float(np.percentile(ends, p)), 1) for p in (50, 90, 99, 99.9)},
                        # drain phase (after the first dry point): wave exits, drain-loop rounds and lane use
                        "exit_after_dry_pct_us": {p: round(float(np.percentile((end - tdry) * tick, p)), 1)
                                                  for p in (10, 25, 50, 75, 90, 99, 100)},
                        "waves_alive_after_dry_us": {t: int(((end - tdry) * tick > t).sum())
                                                     for t in (0, 50, 100, 200, 300, 400, 500)},
                        "drain_rounds_pct": {p: round(float(np.percentile(drounds, p)), 1) for p in (50, 90, 99, 100)},
                        "drain_lane_use": round(float(dlanes.sum() / max(64.0 * drounds.sum(), 1.0)), 3)})
    for o in out:
        print(json.dumps(o))
    r.close()


if __name__ == "__main__":
    main()
