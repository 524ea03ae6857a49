#!/usr/bin/env python3
"""Does a path's ray cost (leaf rounds) predict the cost of its next ray?  Renders the headline
scene at 512x512 @ 8 spp (2^21 paths) with a library built with -DHPT_COST_PROBE
-DHPT_DRAIN_SPLIT=0 (make variant V=cost ..., selected with HAIRPT_LIB) and prints, for each pair of
consecutive trace launches, rank correlations between a path's closest-ray cost at bounce b and
its closest / shadow ray costs at bounce b + 1, and how many of the costliest 5 % of rays at b + 1
a "costly at b" flag (top 30 %) would have put first in the queue.

Usage: HAIRPT_LIB=.../libv_cost/libhairpt.so python tools/cost_probe.py
"""
import ctypes as C
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd"))
import torch  # noqa: E402

from mitsuba_amd import native, scenes  # noqa: E402

L, NP = 6, 1 << 21


def rank(x):
    r = np.empty(len(x))
    r[np.argsort(x, kind="stable")] = np.arange(len(x))
    return r


def spearman(a, b):
    return float(np.corrcoef(rank(a), rank(b))[0, 1])


def main():
    cfg = scenes.CONFIGS["furball_marschner"]
    xml = scenes.make_scene("furball_marschner", os.path.join(tempfile.gettempdir(), "hpt_cost"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": 512, "height": 512, "spp": 8, "maxDepth": cfg["max_depth"]})
    r.prepare()
    lib = native.load_library()
    lib.hpt_debug_costprof.restype = C.c_int
    lib.hpt_debug_costprof.argtypes = [C.c_void_p]
    buf = np.zeros((L, 2, NP), np.uint16)
    film = torch.zeros((512, 512, 4), dtype=torch.float32, device="cuda:0")
    lib.hpt_debug_costprof(buf.ctypes.data)  # clear
    r.render_device(film.data_ptr(), 0, 8)
    torch.cuda.synchronize()
    n = lib.hpt_debug_costprof(buf.ctypes.data)
    print("launches", n)
    for l in range(n):
        c, s = buf[l, 0].astype(np.int64), buf[l, 1].astype(np.int64)
        print("launch %d: closest rays %d mean leaves %.2f p99 %d max %d | shadow rays %d mean %.2f p99 %d max %d" % (
            l, (c > 0).sum(), c[c > 0].mean(), np.percentile(c[c > 0], 99), c.max(),
            (s > 0).sum(), s[s > 0].mean(), np.percentile(s[s > 0], 99), s.max()))
        both = (c > 0) & (s > 0)
        print("   same launch: closest vs shadow cost rank corr %.3f" % spearman(c[both], s[both]))
    for l in range(n - 1):
        c0 = buf[l, 0].astype(np.int64)
        for kind, name in ((0, "closest"), (1, "shadow")):
            c1 = buf[l + 1, kind].astype(np.int64)
            m = (c0 > 0) & (c1 > 0)
            a, b = c0[m], c1[m]
            top = b >= np.percentile(b, 95)
            flag = a >= np.percentile(a, 70)
            print("launch %d -> %d %-7s: rank corr %.3f | costliest 5%% at b+1 flagged costly at b: %.2f (flag rate %.2f)" % (
                l, l + 1, name, spearman(a, b), flag[top].mean(), flag.mean()))
    r.close()


if __name__ == "__main__":
    main()
