#!/usr/bin/env python3
"""Where does k_tail's time go?  Renders rank r of N (default shard 0 of 8) with a
library built with -DHPT_TAIL_PROFILE (make variant V=tailprof KFLAGS=-DHPT_TAIL_PROFILE,
selected with HAIRPT_LIB) and summarises the per-wave timing records of the tail:
iterations (bounces), time in shade / trace / post per iteration (100 MHz ticks), the
longest ray per iteration in leaf rounds, and the wave that finished last.

Usage: HAIRPT_LIB=.../libv_tailprof/libhairpt.so python tools/tail_profile.py [--shards 8]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_tailprof"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                           "maxDepth": cfg["max_depth"]})
    r.prepare()
    lib = native.load_library()
    lib.hpt_debug_tailprof.restype = C.c_int
    lib.hpt_debug_tailprof.argtypes = [C.c_void_p, C.c_int]
    n = 65536
    buf = np.zeros((n, 8), dtype=np.uint64)
    film = torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0")
    spp = cfg["spp"]
    out = {}
    for rep in range(2):
        lib.hpt_debug_tailprof(buf.ctypes.data, n)  # clear
        film.zero_()
        r.render_device(film.data_ptr(), 0, spp, shard=a.shard, n_shards=a.shards, collect_stats=1)
        torch.cuda.synchronize()
        s = r.stats()
        got = lib.hpt_debug_tailprof(buf.ctypes.data, n)
        rec = buf[:got]
        rec = rec[rec[:, 0] > 0]
        it, sh, tr, po, beg, end, rr, live = (rec[:, k].astype(np.float64) for k in range(8))
        t0 = beg.min()
        last = int(np.argmax(end))
        tick = 0.01  # us
        out = {
            "shard": "%d/%d" % (a.shard, a.shards), "tail_ms_event": round(s.ms_tail, 4), "tail_paths": int(s.tail_paths),
            "waves": int(len(rec)), "span_us": round((end.max() - t0) * tick, 1),
            "iterations": {"mean": round(it.mean(), 2), "max": int(it.max()), "p99": float(np.percentile(it, 99))},
            "per_iteration_us_mean": {"shade": round((sh.sum() / it.sum()) * tick, 3),
                                      "trace": round((tr.sum() / it.sum()) * tick, 3),
                                      "post": round((po.sum() / it.sum()) * tick, 3)},
            "rounds_per_iteration_wavemax_mean": round(rr.sum() / it.sum(), 2),
            "last_wave": {"iterations": int(it[last]), "start_us": round((beg[last] - t0) * tick, 1),
                          "end_us": round((end[last] - t0) * tick, 1), "live_lanes_at_start": int(live[last]),
                          "shade_us": round(sh[last] * tick, 1), "trace_us": round(tr[last] * tick, 1),
                          "post_us": round(po[last] * tick, 1), "rounds": int(rr[last]),
                          "us_per_round": round(tr[last] * tick / max(1, rr[last]), 3)},
            "start_spread_us": round((beg.max() - t0) * tick, 1),
        }
        # waves still running over time (a histogram of end times)
        ends = (end - t0) * tick
        out["end_time_percentiles_us"] = {p: round(float(np.percentile(ends, p)), 1) for p in (50, 90, 99, 99.9, 100)}
    print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
