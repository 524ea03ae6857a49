#!/usr/bin/env python3
"""Can a k_trace launch's drain be shortened by claiming predicted-heavy rays first?

Renders rank r of N of the headline frame with a library built with
  make variant V=raylog KFLAGS='-DHPT_RAY_LOG -DHPT_DRAIN_SPLIT=0'
(selected with HAIRPT_LIB), which logs every bounce ray of the first trace launches by work
index (closest rays, then shadow rays): origin, direction, clipped interval length, leaf rounds,
hit flag, path id.  Then, per launch:
  * rank correlation of the true cost (leaf rounds) with cheap predictors known when the ray is
    made: kind, clipped interval length, length inside the hair's bounding sphere, the path's
    previous closest-ray cost;
  * a time-stepped model of the persistent launch (P lanes, one leaf round per step, a step lasts
    max(l0, active lanes / R) us; finished lanes claim the next rays of a claim order) for the
    shipped order (queue order, 64 cursor shards) and for "heavy first" orders: the rays a
    predictor calls light (the lowest fraction f) claimed after all the others, each class in
    queue order over 64 shards; plus the true-cost order as the upper bound.
Prints one JSON line per launch.

Usage: HAIRPT_LIB=.../libv_raylog/libhairpt.so python tools/ray_order_probe.py [--shards 8]
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

LAUNCHES, CAP = 6, 1 << 24
REC = np.dtype([("o", "<f4", 3), ("d", "<f4", 3), ("len", "<f4"), ("cost", "<u4"), ("path", "<u4"), ("pad", "<u4")])
LANES = 7168 * 64          # k_trace's resident lanes (7 waves/SIMD x 1024 SIMDs)
SHARDS = 64


def rank(x):
    r = np.empty(len(x))
    r[np.argsort(x, kind="stable")] = np.arange(len(x))
    return r


def spearman(a, b):
    if len(a) < 3:
        return None
    return round(float(np.corrcoef(rank(a), rank(b))[0, 1]), 3)


def shard_order(idx):
    """claim sequence of the work items idx (in queue order) over 64 contiguous cursor shards that
    advance at the same rate: item j of shard s is claimed at (j - lo_s) / size_s"""
    n = len(idx)
    if n == 0:
        return idx
    j = np.arange(n)
    lo = np.array([(k * n) // SHARDS for k in range(SHARDS + 1)])  # tracePersistent's shard bounds
    s = np.searchsorted(lo, j, side="right") - 1
    sz = np.maximum(lo[s + 1] - lo[s], 1)
    key = (j - lo[s]) / sz
    return idx[np.argsort(key, kind="stable")]


def simulate(order, rounds, l0, R):
    """time-stepped model of the persistent launch; returns (dry time, end time) in us"""
    n = len(order)
    work = rounds[order]
    rem = np.zeros(LANES, dtype=np.int64)
    nxt, t, t_dry = 0, 0.0, None
    while True:
        idle = np.flatnonzero(rem <= 0)
        if nxt < n and len(idle):
            k = min(len(idle), n - nxt)
            rem[idle[:k]] = work[nxt:nxt + k]
            nxt += k
            if nxt >= n and t_dry is None:
                t_dry = t
        active = int((rem > 0).sum())
        if active == 0:
            break
        t += max(l0, active / R)
        rem -= 1
    return (t_dry if t_dry is not None else t), t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--l0", type=float, default=3.0, help="us per leaf round at low load")
    ap.add_argument("--round-us", type=float, default=18.0, help="us per leaf round with every lane busy")
    ap.add_argument("--dump", default="", help="save launches 1 and 3 (cost, lengths, kind, queue order) to this .npz")
    ap.add_argument("--no-sim", action="store_true")
    a = ap.parse_args()
    dump = {}
    cfg = scenes.CONFIGS[a.config]
    xml = scenes.make_scene(a.config, os.path.join(tempfile.gettempdir(), "hpt_raylog"), n_strands=cfg["n"])
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, {"width": cfg["width"], "height": cfg["height"], "spp": cfg["spp"],
                           "maxDepth": cfg["max_depth"]})
    r.prepare()
    info = r.info()
    lo, hi = np.array(info.aabb_min[:3], np.float64), np.array(info.aabb_max[:3], np.float64)
    center, radius = (lo + hi) / 2, float(np.max(hi - lo) / 2)
    lib = native.load_library()
    lib.hpt_debug_raylog.restype = C.c_int
    lib.hpt_debug_raylog.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_uint32]
    bufs = [torch.full((CAP * REC.itemsize,), 255, dtype=torch.uint8, device="cuda:0") for _ in range(LAUNCHES)]
    ptrs = (C.c_void_p * LAUNCHES)(*[b.data_ptr() for b in bufs])
    film = torch.zeros((cfg["height"], cfg["width"], 4), dtype=torch.float32, device="cuda:0")
    lib.hpt_debug_raylog(ptrs, LAUNCHES, CAP)
    r.render_device(film.data_ptr(), 0, cfg["spp"], shard=a.shard, n_shards=a.shards, collect_stats=1)
    torch.cuda.synchronize()
    got = lib.hpt_debug_raylog(ptrs, 0, 0)
    R = LANES / a.round_us
    prev_cost = None
    for li in range(got):
        raw = bufs[li].cpu().numpy().view(REC)
        # the launch's work list: closest rays [0, nTrace) then shadow rays, every one logged
        total = int((raw["path"] != 0xffffffff).sum())
        assert total == 0 or raw["path"][total - 1] != 0xffffffff
        rec = raw[:total]
        cost = (rec["cost"] & 0xffff).astype(np.int64)
        shadow = (rec["cost"] >> 17) & 1
        found = (rec["cost"] >> 16) & 1
        o, d = rec["o"].astype(np.float64), rec["d"].astype(np.float64)
        # length inside the hair's bounding sphere
        oc = o - center
        b = (oc * d).sum(1)
        c = (oc * oc).sum(1) - radius * radius
        disc = b * b - c
        sq = np.sqrt(np.maximum(disc, 0))
        t0, t1 = np.maximum(-b - sq, 0), np.maximum(-b + sq, 0)
        lsph = np.where(disc > 0, t1 - t0, 0.0)
        feats = {"shadow": shadow.astype(np.float64), "len": rec["len"].astype(np.float64), "len_sphere": lsph}
        if prev_cost is not None:
            pc = np.zeros(total)
            m = rec["path"] < len(prev_cost)
            pc[m] = prev_cost[rec["path"][m]]
            feats["prev_closest_cost"] = pc
        rounds = cost + 1
        out = {"launch": li, "rays": total, "closest": int((shadow == 0).sum()), "shadow": int(shadow.sum()),
               "mean_cost": round(float(cost.mean()), 2), "p99": int(np.percentile(cost, 99)), "max": int(cost.max()),
               "spearman": {k: spearman(v, cost) for k, v in feats.items()},
               "spearman_closest": {k: spearman(v[shadow == 0], cost[shadow == 0]) for k, v in feats.items()},
               "spearman_shadow": {k: spearman(v[shadow == 1], cost[shadow == 1]) for k, v in feats.items()}}
        if a.dump and li in (1, 3):
            dump["cost%d" % li] = np.minimum(cost, 255).astype(np.uint8)
            dump["len%d" % li] = rec["len"].astype(np.float16)
            dump["lsph%d" % li] = lsph.astype(np.float16)
            dump["shadow%d" % li] = shadow.astype(np.uint8)
            if "prev_closest_cost" in feats:
                dump["prev%d" % li] = np.minimum(feats["prev_closest_cost"], 255).astype(np.uint8)
        idx = np.arange(total)
        sims = {}
        if a.no_sim:
            print(json.dumps(out), flush=True)
            pcost = np.zeros(int(rec["path"].max()) + 1 if total else 1)
            pcost[rec["path"][shadow == 0]] = cost[shadow == 0]
            prev_cost = pcost
            continue
        dry, end = simulate(shard_order(idx), rounds, a.l0, R)
        sims["queue"] = (dry, end)
        for name, v in list(feats.items()) + [("true_cost", cost.astype(np.float64))]:
            for f in (0.2, 0.35, 0.5):
                light = v <= np.quantile(v, f)
                order = np.concatenate([shard_order(idx[~light]), shard_order(idx[light])])
                sims["%s_f%.2f" % (name, f)] = simulate(order, rounds, a.l0, R)
        base_end = sims["queue"][1]
        out["sim_us"] = {k: {"dry": round(v[0], 1), "drain": round(v[1] - v[0], 1), "end": round(v[1], 1),
                             "saved": round(base_end - v[1], 1)} for k, v in sims.items()}
        print(json.dumps(out), flush=True)
        # the path's closest-ray cost for the next launch's predictor
        pcost = np.zeros(int(rec["path"].max()) + 1 if total else 1)
        cm = shadow == 0
        pcost[rec["path"][cm]] = cost[cm]
        prev_cost = pcost
    if a.dump:
        np.savez_compressed(a.dump, **dump)
    r.close()


if __name__ == "__main__":
    main()
