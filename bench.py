#!/usr/bin/env python3
"""Headline benchmark: Mpaths/s of the hair path tracer on MI355X.

Workload (BASELINE.json configs[2], the metric's config): models/furball with
the Marschner BSDF, 512x512 @ 256 spp, maxDepth 65, synthetic furball hair
(40,000 strands, ~3.2e5 segments, seed 1), sunsky stand-in lighting.
One step = one full frame: every sample of every pixel traced to
termination (MIPathTracer::Li, path.cpp:119-294) and splatted into the film.
With N GPUs the frame's 32x32 blocks are dealt cyclically along a Hilbert curve to ranks and
the RGBW films are summed on rank 0 with one RCCL reduce (strong scaling).

Launch:  python bench.py [--gpus 1 --steps 3 --warmup 1]
         python bench.py --gpus N ...   (starts the N ranks itself: a child torch.distributed.run)
         python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Prints ONE JSON line on rank 0.  --gpus must equal WORLD_SIZE when a launcher set it.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (import first: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from mitsuba_amd import distributed, native, scenes  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

# Algorithmic bytes of the traversal kernels.
# roofline.achieved uses SURVEY.md 8(d)'s per-unit model: 8 B per binary kd-node visit, 4 B leaf
# index + 52 B primitive per primitive test, plus the ray's own I/O:
#   closest ray: queue id 4 + ray 32 + hit record 16 (segment, t, root) = 52 B
#   shadow ray:  queue id 4 + origin 16 + direction/maxt 16 = 36 B, +48 B (contribution + radiance RMW)
#                when unoccluded
BYTES_CLOSEST, BYTES_SHADOW, BYTES_UNOCC = 52, 36, 48
B8D_NODE, B8D_REF, B8D_PRIM = 8, 4, 52
# the layout-specific figure (what this build's records actually are): 32 B per two-level HptNode4
# fetch, 16 B leaf-ordered fp32 pre-test record (HptSegQ) per primitive test, 128 B segment record
# per exact fp64 test; the packet pass reads 8-byte binary HptNodes and 32-byte HptSegF records
BYTES_NODE4, BYTES_PRIM, BYTES_EXACT, BYTES_NODE2, BYTES_PRIM_PACKET = 32, 16, 128, 8, 32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="furball_marschner")
    ap.add_argument("--strands", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--max-depth", type=int, default=None)
    ap.add_argument("--kd", default="", help="kd-tree build overrides k=v,... (hair shape kd* properties)")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-spp", type=int, default=96, help="spp of the bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = the CPUs this process can actually use: min(affinity CPUs, cgroup CPU quota)")
    ap.add_argument("--cpu-nproc-run", choices=["auto", "off"], default="auto",
                    help="also time the sample on one thread per affinity CPU (nproc, SURVEY.md 8(d)) when that "
                         "differs from the effective CPUs")
    ap.add_argument("--balance", choices=["on", "off"], default="on",
                    help="N > 1: after the warm-up, re-deal the blocks by the work each shaded (path-bounces "
                         "summed over ranks, hpt_set_block_weights); off: the Hilbert-cyclic deal")
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "hpt_bench"))
    return ap.parse_args()


def cpu_baseline(args, cfg, xml_defines, hair_src, env_rgb, nodes, idx):
    """Oracle built with the reference's flags (liboracle_ref.so), bounded sample on host cores."""
    import oracle_lib
    import scene_util

    _, cam, _ = scene_util.config_params(args.config)
    o = oracle_lib.Oracle(variant="ref")
    W, H = xml_defines["width"], xml_defines["height"]
    env_rgb = scene_util.oracle_envmap(args.config) if env_rgb is None else env_rgb
    o.setup(cam, 35.0, W, H, scene_util.oracle_shapes(args.config, hair_src[1], hair_src[0]), None, None, env_rgb,
            xml_defines["maxDepth"])
    o.set_kdtree(nodes, idx)
    o.prepare()
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None  # the cgroup's CPU bandwidth limit (cgroup v2 cpu.max "quota period"), in CPUs
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    # the CPUs the process can actually use: the affinity set, capped by the cgroup quota (on the
    # GPU box 256 affinity CPUs share a 16-CPU quota: 256 threads are time-sliced onto 16)
    effective = max(1, min(avail, int(quota))) if quota else avail
    threads = args.cpu_threads if args.cpu_threads > 0 else effective
    paths = W * H * args.cpu_spp

    def timed(n_threads):
        t0 = time.perf_counter()
        o.render(0, args.cpu_spp, threads=n_threads, width=W, height=H)
        return time.perf_counter() - t0

    dt = timed(threads)
    nproc_run = None
    if args.cpu_nproc_run == "auto" and avail != threads:
        dn = timed(avail)
        nproc_run = {"value": paths / dn / 1e6, "threads": avail,
                     "note": "one worker per affinity CPU (nproc, like mitsuba.cpp:135,281), time-sliced onto "
                             "the cgroup quota"}
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), model)
    except OSError:
        pass
    return {"value": paths / dt / 1e6, "unit": "Mpaths/s", "cores": min(threads, effective), "threads": threads,
            "kind": "port", "cpu_model": model, "host_cpus": os.cpu_count(), "affinity_cpus": avail,
            "cgroup_cpu_quota": quota,
            "cores_note": "cores = the CPUs the run could use, min(threads, affinity CPUs, cgroup quota)",
            "nproc_run": nproc_run,
            "sample": "%dx%d @ %d spp of the same scene (%d paths), %.2f s, liboracle_ref.so "
                      "(-O3 -march=nocona -msse2 -funsafe-math-optimizations, config-ubuntu-20.04.py:8; "
                      "the oracle adds -ftree-vectorize -ffp-contract=off and traverses the product's kd-tree)"
                      % (W, H, args.cpu_spp, paths, dt)}


def timed_steps(step, steps, world, dist_mod, sync, device, after_step=None):
    """Time exactly `steps` calls of step(), bracketed by a barrier + device sync on both
    sides; returns the MAX over ranks of the elapsed seconds (the driver's contract).
    Covered on the CPU by tests/test_distributed.py (gloo, world size 2)."""
    if world > 1:
        dist_mod.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        if after_step is not None:
            after_step()
    sync()
    if world > 1:
        dist_mod.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    if world > 1:
        dist_mod.all_reduce(t, op=dist_mod.ReduceOp.MAX)
    return float(t.item())


def launch_ranks(n_ranks, argv):
    """`bench.py --gpus N` without a launcher: run the N ranks as a CHILD torch.distributed.run
    (one process per GPU; this parent has made no HIP call, and it does not exec: it waits for
    the child and returns its exit code).  The ranks inherit stdout, so rank 0's one JSON line
    is this command's output.  One command drives every worker, as mitsuba.cpp:281-329 does."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n_ranks),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def check_world(gpus, env):
    """The rank count the launcher gave (WORLD_SIZE) must be the --gpus asked for: a line that says
    n_gpus N must have run N ranks.  Returns the world size; raises SystemExit on a mismatch."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if gpus != 1:
            raise SystemExit("bench.py: --gpus %d needs %d ranks; run it without a launcher (it starts them) or under "
                             "torch.distributed.run --nproc-per-node %d" % (gpus, gpus, gpus))
        return 1
    if int(ws) != gpus:
        raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%s ranks" % (gpus, ws))
    return int(ws)


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = check_world(args.gpus, os.environ)
    rank = int(os.environ.get("RANK", "0"))
    # HPT_BENCH_BACKEND=gloo only rehearses N > 1 on a one-GPU box (RCCL refuses two
    # ranks on one device): the film is reduced from a host copy.  Never the bench.
    backend = os.environ.get("HPT_BENCH_BACKEND", "nccl")
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_dev = max(1, torch.cuda.device_count())
    if backend == "gloo":
        local %= n_dev  # the rehearsal's ranks share the visible devices
    elif local >= n_dev:
        raise SystemExit("LOCAL_RANK %d but only %d visible GPU(s): one rank per GPU (HIP_VISIBLE_DEVICES too narrow?)"
                         % (local, n_dev))
    pg = {"dist_backend": None, "world_size": 1, "rccl_version": None}
    if world > 1:
        dist.init_process_group(backend)  # "nccl" = RCCL over xGMI on ROCm
        # what the process group itself reports (not the launcher's environment)
        pg["dist_backend"] = str(dist.get_backend())
        pg["world_size"] = dist.get_world_size()
        if pg["world_size"] != world:
            raise SystemExit("bench.py: the process group has %d ranks, WORLD_SIZE says %d" % (pg["world_size"], world))
        if pg["dist_backend"] == "nccl":
            try:
                import torch.cuda.nccl as tnccl
                pg["rccl_version"] = ".".join(str(v) for v in tnccl.version())
            except Exception as ex:  # noqa: BLE001 -- a version we cannot read is recorded as such
                pg["rccl_version"] = "unknown (%s)" % type(ex).__name__
    torch.cuda.set_device(local)
    cfg = scenes.CONFIGS[args.config]
    n = args.strands or cfg["n"]
    W = args.width or cfg["width"]
    H = args.height or cfg["height"]
    spp = args.spp or cfg["spp"]
    max_depth = args.max_depth if args.max_depth is not None else cfg["max_depth"]
    defines = {"width": W, "height": H, "spp": spp, "maxDepth": max_depth}
    workdir = os.path.join(args.workdir, "r%d" % rank)
    xml = scenes.make_scene(args.config, workdir, n_strands=n)
    if args.kd:
        xml = scenes.with_kd_params(xml, dict(kv.split("=") for kv in args.kd.split(",") if kv))
    hair_src = (workdir, n)  # the oracle re-reads the same hair file(s)

    r = native.Renderer(device=local)
    r.load_scene_xml(xml, defines)
    t0 = time.perf_counter()
    r.prepare()
    t_prep = time.perf_counter() - t0
    info = r.info()
    film = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda:%d" % local)
    host_film = torch.zeros((H, W, 4), dtype=torch.float32) if backend == "gloo" else None

    def step(level):
        film.zero_()
        torch.cuda.synchronize()
        if host_film is None:
            distributed.render_frame(
                lambda shard, n_shards, f: r.render_device(f.data_ptr(), 0, spp, shard=shard, n_shards=n_shards,
                                                            collect_stats=level),
                film, rank, world, dist)
        else:
            def shard_to_host(shard, n_shards, f):
                r.render_device(film.data_ptr(), 0, spp, shard=shard, n_shards=n_shards, collect_stats=level)
                f.copy_(film)
            distributed.render_frame(shard_to_host, host_film, rank, world, dist)
            film.copy_(host_film)

    n_blocks = ((W + 31) // 32) * ((H + 31) // 32)
    balance = world > 1 and args.balance == "on"
    for i in range(args.warmup):
        if balance and i == args.warmup - 1:
            r.block_costs(n_blocks)  # read and reset: the counts balance_blocks reads cover one frame
        step(1)
    balanced = False
    if balance:
        # the last warm-up frame's per-block path-bounces, summed over the ranks, deal the blocks
        # longest-first (the same deal on every rank); one more frame records its schedules
        distributed.balance_blocks(r, n_blocks, world, dist, "cuda:%d" % local if backend == "nccl" else "cpu",
                                   spp=spp, width=W, height=H, frames=1)
        step(1)
        balanced = True
    # one untimed counted frame: traversal counters for the byte model (the
    # render is deterministic, so every frame has exactly these counts)
    step(2)
    c = r.stats()
    frame = dict(nodes=c.nodes, bnodes=c.binary_nodes, prims=c.prims, exact=c.prim_exact, closest=c.closest_rays, shadow=c.shadow_rays,
                 unocc=c.shadow_unoccluded, bounces=c.bounces, launches=c.trace_launches,
                 node_slots=c.node_slots, prim_slots=c.prim_slots,
                 p_rays=c.packet_rays, p_nodes=c.packet_nodes, p_prims=c.packet_prims, p_exact=c.packet_exact,
                 p_node_slots=c.packet_node_slots, p_prim_slots=c.packet_prim_slots, p_fallbacks=c.packet_fallbacks)
    acc = {"ms_trace": 0.0, "ms_packet": 0.0, "launches": 0, "p_launches": 0, "kernels": {}}

    def collect():
        # HIP events (on the library's stream) around the traversal launches only (collect_stats 3):
        # an event around every kernel costs the frame ~4 us per event between launches
        s = r.stats()
        acc["ms_trace"] += s.ms_trace
        acc["launches"] += s.trace_launches
        acc["ms_packet"] += s.ms_trace_packet
        acc["p_launches"] += s.packet_launches

    dt = timed_steps(lambda: step(3), args.steps, world, dist, torch.cuda.synchronize, "cuda:%d" % local, collect)
    # the per-kernel split, averaged over three more (untimed) frames with an event around every
    # kernel (the timed steps carry events around the traversal launches only: collect_stats 3)
    split_frames = 3
    for _ in range(split_frames):
        step(1)
        s1 = r.stats()
        for k in ("camera", "trace_packet", "trace", "primary", "shade", "post", "tail", "gather"):
            acc["kernels"][k] = acc["kernels"].get(k, 0.0) + getattr(s1, "ms_" + k) / split_frames
    # the same frame once more with no recorded bounce schedule (what a render of a new spp range
    # or the CLI's first pass does: every bounce's queue length read back); not
    # part of `value`, which times repeated frames of the same spp range
    r.clear_schedules()
    first_ms = 1e3 * timed_steps(lambda: step(1), 1, world, dist, torch.cuda.synchronize, "cuda:%d" % local)
    assert r.stats().waves_ahead == 0
    ms_trace, ms_packet, launches, p_launches = acc["ms_trace"], acc["ms_packet"], acc["launches"], acc["p_launches"]
    ms_kernels = acc["kernels"]
    tot = {k: v * args.steps for k, v in frame.items()}

    workload = "%s %dx%d @ %d spp, maxDepth %d, %d strands / %d segments" % (
        args.config, W, H, spp, max_depth, n, info.segments)
    paths_total = W * H * spp * args.steps
    value = paths_total / dt / 1e6
    io = BYTES_CLOSEST * tot["closest"] + BYTES_SHADOW * tot["shadow"] + BYTES_UNOCC * tot["unocc"]
    bytes_alg = io + B8D_NODE * tot["bnodes"] + (B8D_REF + B8D_PRIM) * tot["prims"]
    bytes_lay = io + BYTES_NODE4 * tot["nodes"] + BYTES_PRIM * tot["prims"] + BYTES_EXACT * tot["exact"]
    gbs = lambda b, ms: b / (ms * 1e-3) / 1e9 if ms > 0 else 0.0  # noqa: E731
    achieved, achieved_lay = gbs(bytes_alg, ms_trace), gbs(bytes_lay, ms_trace)
    # the packet pass reads a node or a leaf record once per PACKET step (wave-uniform scalar
    # loads), so 8(d)'s per-unit figures are charged per step (slots / 64), not per member
    # lane; each lane still reads and writes its own ray (52 B)
    io_pk = BYTES_CLOSEST * tot["p_rays"]
    pk_node_steps, pk_prim_steps = tot["p_node_slots"] / 64.0, tot["p_prim_slots"] / 64.0
    bytes_pk = io_pk + B8D_NODE * pk_node_steps + (B8D_REF + B8D_PRIM) * pk_prim_steps
    bytes_pk_lane = io_pk + B8D_NODE * tot["p_nodes"] + (B8D_REF + B8D_PRIM) * tot["p_prims"]
    bytes_pk_lay = io_pk + BYTES_NODE2 * pk_node_steps + BYTES_PRIM_PACKET * pk_prim_steps + BYTES_EXACT * tot["p_exact"]
    achieved_pk, achieved_pk_lay = gbs(bytes_pk, ms_packet), gbs(bytes_pk_lay, ms_packet)
    # the whole frame on SURVEY.md 8(d)'s B_path: camera ray + state 40 B per path; per path-bounce
    # the state queue read + write 2 x 80, the hit record 40, the BSDF's table reads (Marschner
    # ~430 B, Kajiya-Kay 0) and NEE's envmap reads 108; per shadow ray its record 80; every
    # traversal at 8 B per binary node + 56 B per primitive test (camera rays per lane); the film
    # gather 9 x 16 B read + 16 B written per pixel
    b_bsdf = 430 if "marschner" in args.config else 0
    bytes_frame = (40 * paths_total + (2 * 80 + 40 + b_bsdf + 108) * tot["bounces"] + 80 * tot["shadow"]
                   + bytes_alg - io + B8D_NODE * tot["p_nodes"] + (B8D_REF + B8D_PRIM) * tot["p_prims"]
                   + (9 * 16 + 16) * W * H * args.steps)
    achieved_frame = bytes_frame / dt / 1e9
    traffic, traffic_src, traffic_pk, limiter = None, None, None, None
    tj = os.path.join(ROOT, "profiles", "traffic_%s.json" % args.config)
    if os.path.exists(tj):
        # HBM-side bytes per k_trace launch from the committed rocprofv3 PMC passes
        # (scripts/gpu_profile.sh + tools/rocpd_summary.py) of this same workload
        t = json.load(open(tj))
        if t.get("workload") == workload and "k_trace" in t.get("kernels", {}):
            traffic = round(t["kernels"]["k_trace"]["bytes_per_launch"])
            traffic_src = "profiles/" + os.path.basename(tj)
            if "k_trace_packet" in t["kernels"]:
                traffic_pk = round(t["kernels"]["k_trace_packet"]["bytes_per_launch"])
            limiter = t.get("limiter")
    out = None
    if rank == 0:
        cpu = None
        if args.cpu_baseline == "auto" and world == 1:
            nodes, idx, _ = r.kdtree()
            cpu = cpu_baseline(args, cfg, defines, hair_src, None, nodes, idx)
        img = native.develop(film.cpu().numpy())
        out = {
            "metric": "Mpaths/sec + achieved HBM GB/s, furball Marschner 512² @ 256spp",
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32 (f64 cylinder tests)",
            "data": "synthetic hair (seeded, BINARY_HAIR; reference hair blobs absent) lit by the scene's sunsky (Hosek-Wilkie sky + Preetham sun rasterised like sunsky.cpp)",
            "config": {"workload": workload,
                       "paths_per_step": W * H * spp, "parallelism": "tiles%d" % world,
                       "gpus_arg": args.gpus, **pg,
                       "deal": "work-balanced (warm-up frame's path-bounces per block)" if balanced
                       else "Hilbert-cyclic 32x32 blocks",
                       **({"rehearsal": "HPT_BENCH_BACKEND=gloo: ranks share GPUs, host-copy reduce"}
                          if host_film is not None and world > 1 else {}),
                       "kd_nodes": int(info.kd_nodes), "kd_depth": int(info.kd_depth),
                       "prepare_s": round(t_prep, 3)},
            # bound: the roofline the kernel is priced against (HBM: no dense contraction here);
            # limiter: what the PMC counters say actually holds it below that roofline
            "roofline": {"bound": "hbm", "limiter": limiter, "kernel": "k_trace", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_calibration": "profiles/r03_fetch_calibration.json: FETCH_SIZE is 64 B per 128-B "
                                                "line for 8/16/32-B accesses, cold or Infinity-Cache resident (x2 = "
                                                "line bytes); WRITE_SIZE is 32 B per lone 16-B store",
                         "achieved_hbm": round(traffic / (ms_trace / max(1, launches)) * 1e-6, 1)
                         if traffic and ms_trace > 0 else None,
                         "frac_hbm": round(traffic / (ms_trace / max(1, launches)) * 1e-6 / HBM_PEAK_GBS, 4)
                         if traffic and ms_trace > 0 else None,
                         "algorithmic_model": "SURVEY.md 8(d): 8 B per binary kd-node visit, 4+52 B per primitive "
                                              "test, ray I/O 52 (closest) / 36 (+48 unoccluded) B; the closest "
                                              "ray's hit record is priced at 8(d)'s 16 B (segment, t, root), "
                                              "while the product writes a 4-B hit word",
                         "algorithmic_bytes_per_launch": int(bytes_alg // max(1, launches)),
                         "achieved_layout": round(achieved_lay, 1),
                         "layout_bytes_per_launch": int(bytes_lay // max(1, launches)),
                         "avg_launch_ms": round(ms_trace / max(1, launches), 4), "launches": int(launches),
                         "bytes_per_step": int(bytes_alg // args.steps),
                         "rank0_trace_ms_per_step": round(ms_trace / args.steps, 3)},
            # the camera pass's packet traversal (k_trace_packet): 8(d) bytes per packet step
            "roofline_packet": {"bound": "hbm", "kernel": "k_trace_packet", "achieved": round(achieved_pk, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved_pk / HBM_PEAK_GBS, 4),
                                "traffic": traffic_pk,
                                "achieved_hbm": round(traffic_pk / (ms_packet / max(1, p_launches)) * 1e-6, 1)
                                if traffic_pk and ms_packet > 0 else None,
                                "algorithmic_model": "SURVEY.md 8(d) per packet step: 8 B per binary-node step, "
                                                     "4+52 B per leaf-record step (wave-uniform), 52 B ray I/O per lane",
                                "algorithmic_bytes_per_launch": int(bytes_pk // max(1, p_launches)),
                                "lane_demand_bytes_per_launch": int(bytes_pk_lane // max(1, p_launches)),
                                "achieved_layout": round(achieved_pk_lay, 1),
                                "avg_launch_ms": round(ms_packet / max(1, p_launches), 4),
                                "launches": int(p_launches)},
            # every kernel of the frame on the same byte model, over the whole timed step
            "roofline_frame": {"bound": "hbm", "achieved": round(achieved_frame, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(achieved_frame / HBM_PEAK_GBS, 4),
                               "bytes_per_step": int(bytes_frame // args.steps),
                               "algorithmic_model": "SURVEY.md 8(d) B_path summed over the frame: camera 40 B/path; "
                                                    "per path-bounce 2x80 state + 40 hit + BSDF tables (%d) + NEE 108; "
                                                    "80 B per shadow ray; traversal 8 B/binary node, 56 B/primitive "
                                                    "test (camera rays per lane); film 160 B/pixel" % b_bsdf},
            # value times repeated frames of one spp range, whose bounces are launched ahead on the
            # schedule recorded by the first render; this is that first render (one frame)
            "first_render_ms": round(first_ms, 3),
            "kernel_ms_per_step": {k: round(v, 3) for k, v in ms_kernels.items()},
            "timing": "timed steps: HIP events around the traversal launches only (collect_stats 3); "
                      "kernel_ms_per_step: the mean of three more frames with an event around every kernel",
            "cpu_baseline": cpu,
            "stats": {"bounces_per_path": round(tot["bounces"] / max(1, paths_total / world), 4),
                      "nodes_per_ray": round(tot["nodes"] / max(1, tot["closest"] + tot["shadow"]), 2),
                      "binary_nodes_per_ray": round(tot["bnodes"] / max(1, tot["closest"] + tot["shadow"]), 2),
                      "prims_per_ray": round(tot["prims"] / max(1, tot["closest"] + tot["shadow"]), 2),
                      "exact_tests_per_ray": round(tot["exact"] / max(1, tot["closest"] + tot["shadow"]), 2),
                      "simd_util_nodes": round(tot["nodes"] / max(1, tot["node_slots"]), 3),
                      "simd_util_prims": round(tot["prims"] / max(1, tot["prim_slots"]), 3),
                      "camera_rays_packet": int(frame["p_rays"]),
                      "camera_binary_nodes_per_ray": round(tot["p_nodes"] / max(1, tot["p_rays"]), 2),
                      "camera_prims_per_ray": round(tot["p_prims"] / max(1, tot["p_rays"]), 2),
                      "camera_packet_util_nodes": round(tot["p_nodes"] / max(1, tot["p_node_slots"]), 3),
                      "camera_packet_util_prims": round(tot["p_prims"] / max(1, tot["p_prim_slots"]), 3),
                      "camera_packet_fallbacks": int(frame["p_fallbacks"]),
                      "image_mean": float(img.mean()),
                      # exact-arithmetic fingerprint of the frame (sum of the RGBW film in fp64):
                      # identical for every traversal variant, since hits are bit-exact
                      "film_fingerprint": float(film.double().sum().item())},
        }
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
