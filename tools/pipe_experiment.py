#!/usr/bin/env python3
"""Experiment: can two render calls on one GPU (two contexts, two streams, two host
threads) overlap each other's launch drains?  Times one N-shard frame rendered by one
context vs the same frame split by spp over two contexts running concurrently."""
import argparse
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd"))
import torch  # noqa: E402
from mitsuba_amd import native, scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_pipe"), n_strands=cfg["n"])
    rs = []
    for _ in range(2):
        r = native.Renderer(device=0)
        r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                               "maxDepth": cfg["max_depth"]})
        r.prepare()
        rs.append(r)
    films = [torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0") for _ in range(2)]
    spp = cfg["spp"]
    for n in sorted({1, a.n}):
        def single():
            rs[0].render_device(films[0].data_ptr(), 0, spp, shard=0, n_shards=n)

        def split():
            ths = [threading.Thread(target=lambda k=k: rs[k].render_device(films[k].data_ptr(), k * spp // 2,
                                                                           (k + 1) * spp // 2, shard=0, n_shards=n))
                   for k in range(2)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()

        for name, fn in (("single", single), ("split2", split)):
            fn()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            print("N=%d shard 0 %-7s %.2f ms (HPT_PERSIST_FRAC=%s)" % (n, name, best * 1e3,
                                                                       os.environ.get("HPT_PERSIST_FRAC", "1")),
                  flush=True)


if __name__ == "__main__":
    main()
