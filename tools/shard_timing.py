#!/usr/bin/env python3
"""Single-GPU rehearsal of bench.py's strong scaling: time the frame share of
rank r of N (block-cyclic shards, hpt_render_device shard=r, n_shards=N) on
one GPU, for N = 1, 2, 4, 8.  The slowest rank bounds a multi-GPU frame, so
max over r of these times (plus one 4 MB RCCL reduce) is what bench.py
--gpus N measures per step.

Usage: python tools/shard_timing.py [--config furball_marschner] [--reps 3] [--all-ranks]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd"))

import torch  # noqa: E402

from mitsuba_amd import native, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--all-ranks", action="store_true", help="time every rank of each N (default: rank 0 and the slowest of a sample)")
    ap.add_argument("--ns", default="2,4,8", help="shard counts to time (besides N=1)")
    ap.add_argument("--split", choices=["blocks", "spp"], default="blocks",
                    help="rank r of N: its Hilbert-cyclic blocks (bench.py) or spp range [r*spp/N, (r+1)*spp/N) of every pixel")
    ap.add_argument("--balance", nargs="?", const="camera", choices=["bounces", "camera"],
                    help="deal the blocks by the work each did in a first frame (hpt_set_block_weights): its "
                         "path-bounces, or those plus its camera rays (bench.py's deal, the default)")
    ap.add_argument("--stats-level", type=int, default=0,
                    help="hpt_render_params.collect_stats of the timed renders (0: no events between launches; the "
                         "per-kernel split comes from one more render of the shard at level 1)")
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_shards"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                           "maxDepth": cfg["max_depth"]})
    r.prepare()
    film = torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0")
    spp = cfg["spp"]

    def timed(shard, n):
        best = 1e30
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if a.split == "spp":
                r.render_device(film.data_ptr(), shard * spp // n, (shard + 1) * spp // n, collect_stats=a.stats_level)
            else:
                r.render_device(film.data_ptr(), 0, spp, shard=shard, n_shards=n, collect_stats=a.stats_level)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        if a.stats_level == 0:  # the per-kernel split, from one more (untimed) render with events
            if a.split == "spp":
                r.render_device(film.data_ptr(), shard * spp // n, (shard + 1) * spp // n, collect_stats=1)
            else:
                r.render_device(film.data_ptr(), 0, spp, shard=shard, n_shards=n, collect_stats=1)
            torch.cuda.synchronize()
        return best, r.stats()

    r.render_device(film.data_ptr(), 0, spp)  # warm-up
    if a.balance:  # every block's measured work, as bench.py's ranks sum it
        nb = ((cfg["width"] + 31) // 32) * ((cfg["height"] + 31) // 32)
        from mitsuba_amd import distributed
        costs = r.block_costs(nb).astype("float64")
        r.set_block_weights(costs if a.balance == "bounces" else
                            distributed.block_weights(costs, spp, cfg["width"], cfg["height"]))
    t1, _ = timed(0, 1)
    out = {"config": a.config, "N1_ms": round(t1 * 1e3, 3), "shards": {}}
    for n in [int(x) for x in a.ns.split(",")]:
        ranks = range(n) if a.all_ranks else sorted({0, n - 1})
        ts, work = {}, {}
        for k in ranks:
            t, s = timed(k, n)
            ts[k] = (round(t * 1e3, 3), round(s.ms_trace, 3), round(s.ms_tail, 3))
            work[k] = (int(s.bounces), int(s.paths), round(s.ms_trace_packet, 3))
            if k == 0:
                kern = {n: round(getattr(s, "ms_" + n), 3) for n in
                        ("camera", "trace_packet", "primary", "trace", "shade", "post", "tail", "gather")}
                print("N=%d rank 0 kernels (ms): %s; sum %.2f of %.2f wall" % (n, kern, sum(kern.values()), t * 1e3),
                      flush=True)
        worst = max(v[0] for v in ts.values())
        out["shards"][n] = {"per_rank_ms_trace_tail": ts, "per_rank_bounces_paths_packet_ms": work, "max_ms": worst,
                            "efficiency": round(t1 * 1e3 / (n * worst), 4)}
        print("N=%d ranks %s -> max %.2f ms, strong-scaling efficiency %.3f" % (n, ts, worst, t1 * 1e3 / (n * worst)),
              flush=True)
    print(json.dumps(out))
    r.close()


if __name__ == "__main__":
    main()
