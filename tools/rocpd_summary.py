#!/usr/bin/env python3
"""Summarise rocprofv3 rocpd databases (kernel trace + FETCH_SIZE/WRITE_SIZE
passes written by scripts/gpu_profile.sh) into a committed text summary.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM / rocprofv3):
FETCH_SIZE (KiB) reports half the bytes of wide streaming reads on gfx950, so
it is doubled; WRITE_SIZE (KiB) is taken as is.  Both count fabric-side L2
requests (Infinity-Cache hits included)."""
import argparse
import glob
import os
import sqlite3


def one_db(d):
    f = glob.glob(os.path.join(d, "*.db"))
    if not f:
        raise SystemExit("no rocpd db under %s" % d)
    return sqlite3.connect(f[0])


def fmt(x, digits=2):
    if x is None:
        return "-"
    return ("%%.%df" % digits) % x


def pmc_summary(d):
    """per kernel: counter sums over every launch, from every group database under d"""
    sums = {}
    for g in sorted(glob.glob(os.path.join(d, "g*"))):
        if not os.path.isdir(g):
            continue
        try:
            db = one_db(g)
        except SystemExit:
            continue
        for kn, ctr, val in db.execute("select kernel_name, counter_name, sum(value) from counters_collection "
                                       "group by kernel_name, counter_name"):
            sums.setdefault(kn, {})[ctr] = val
        # the kernel's summed launch durations (ns) in the pass that counted SQ_INSTS_SALU
        for kn, dur in db.execute("select kernel_name, sum(duration) from counters_collection "
                                  "where counter_name='SQ_INSTS_SALU' group by kernel_name"):
            sums.setdefault(kn, {})["_salu_pass_ns"] = dur
    out = {}
    for kn, c in sums.items():
        cyc = c.get("SQ_WAVE_CYCLES")
        waves = c.get("SQ_WAVES")
        r = {}
        if cyc:
            r["wait"] = c.get("SQ_WAIT_ANY", 0) / cyc
            r["inst_wait"] = c.get("SQ_WAIT_INST_ANY", 0) / cyc
            r["valu"] = c.get("SQ_ACTIVE_INST_VALU", 0) / cyc
        if c.get("TCC_HIT_sum") is not None and c.get("TCC_MISS_sum") is not None:
            r["l2_hit"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
            r["l1_miss"] = c.get("TCP_TCC_READ_REQ_sum", 0) / c["TCP_TOTAL_CACHE_ACCESSES_sum"]
        if waves:
            r["vmem_per_wave"] = c.get("SQ_INSTS_VMEM_RD", 0) / waves
            r["lds_per_wave"] = c.get("SQ_INSTS_LDS", 0) / waves
            r["salu_per_wave"] = c.get("SQ_INSTS_SALU", 0) / waves
            r["valu_per_wave"] = c.get("SQ_INSTS_VALU", 0) / waves
        if c.get("_salu_pass_ns"):
            # the CU's one scalar unit issues at most one instruction per cycle (MI355X_MICROARCH.md:
            # 4 SIMDs, 1 scalar unit per CU): SALU instructions per CU-cycle at 2.4 GHz over 256 CUs
            r["salu_issue"] = c.get("SQ_INSTS_SALU", 0) / (c["_salu_pass_ns"] * 2.4 * 256)
        r["counters"] = c
        out[kn] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir", help="gpurun_out/prof_<tag> (trace/, fetch/, write/)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    ap.add_argument("--json", default=None, help="also write per-launch traffic as JSON (read by bench.py)")
    ap.add_argument("--workload", default="", help="workload string the traffic belongs to (bench config)")
    ap.add_argument("--pmc", default=None, help="gpurun_out/pmc_<tag> (g1..gN from scripts/gpu_pmc.sh)")
    a = ap.parse_args()
    lines = []
    if a.title:
        lines += ["# " + a.title, ""]
    db = one_db(os.path.join(a.prof_dir, "trace"))
    lines.append("## rocprofv3 --kernel-trace --stats (durations in microseconds)")
    lines.append("")
    lines.append("| kernel | calls | total_us | avg_us | % |")
    lines.append("|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in db.execute("select name, total_calls, total_duration, average, percentage "
                                                 "from top_kernels"):
        name = name if len(name) < 60 else name[:57] + "..."
        lines.append("| %s | %d | %.1f | %.1f | %.2f |" % (name, calls, tot, avg, pct))
    traffic = {}
    for tag, ctr in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        p = os.path.join(a.prof_dir, tag)
        if not os.path.isdir(p):
            continue
        d = one_db(p)
        for kn, n, s, dur in d.execute("select kernel_name, count(*), sum(value), avg(duration) from "
                                       "counters_collection where counter_name=? group by kernel_name", (ctr,)):
            traffic.setdefault(kn, {})[ctr] = (n, s, dur)
    if traffic:
        lines += ["", "## HBM-side traffic per launch (separate --pmc passes)", "",
                  "| kernel | launches | FETCH_SIZE x2 (MB/launch) | WRITE_SIZE (MB/launch) | total (MB/launch) |",
                  "|---|---:|---:|---:|---:|"]
        for kn, v in sorted(traffic.items(), key=lambda kv: -kv[1].get("FETCH_SIZE", (1, 0, 0))[1]):
            f = v.get("FETCH_SIZE", (1, 0.0, 0))
            w = v.get("WRITE_SIZE", (1, 0.0, 0))
            fm = 2.0 * f[1] * 1024 / max(1, f[0]) / 1e6
            wm = w[1] * 1024 / max(1, w[0]) / 1e6
            if fm + wm < 0.01:
                continue
            kn = kn if len(kn) < 60 else kn[:57] + "..."
            lines.append("| %s | %d | %.1f | %.1f | %.1f |" % (kn, f[0], fm, wm, fm + wm))
    pmc = pmc_summary(a.pmc) if a.pmc else {}
    if pmc:
        lines += ["", "## Occupancy / stall / cache counters (scripts/gpu_pmc.sh, one rocprofv3 --pmc pass per group)",
                  "", "Ratios of counters summed over all launches of the kernel: wait = SQ_WAIT_ANY / "
                  "SQ_WAVE_CYCLES (wave-cycles parked on a dependency, mostly memory), valu = "
                  "SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, inst-wait = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, "
                  "L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS), L1 miss to L2 = TCP_TCC_READ_REQ / "
                  "TCP_TOTAL_CACHE_ACCESSES, SALU issue = SQ_INSTS_SALU per CU-cycle (2.4 GHz, 256 CUs; the "
                  "CU's one scalar unit issues at most one per cycle).", "",
                  "| kernel | wait | inst-wait | valu | L2 hit | L1->L2 reads | VMEM rd / wave | LDS inst / wave "
                  "| SALU inst / wave | VALU inst / wave | SALU issue |",
                  "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
        for kn in ("k_trace", "k_trace_packet", "k_shade", "k_post", "k_tail", "k_camera", "k_primary"):
            v = pmc.get(kn)
            if not v:
                continue
            lines.append("| %s | %s | %s | %s | %s | %s | %s | %s | %s | %s | %s |" % (
                kn, fmt(v.get("wait")), fmt(v.get("inst_wait")), fmt(v.get("valu")), fmt(v.get("l2_hit")),
                fmt(v.get("l1_miss")), fmt(v.get("vmem_per_wave"), 0), fmt(v.get("lds_per_wave"), 0),
                fmt(v.get("salu_per_wave"), 0), fmt(v.get("valu_per_wave"), 0), fmt(v.get("salu_issue"))))
    open(a.out, "w").write("\n".join(lines) + "\n")
    if a.json:
        import json

        out = {"workload": a.workload, "source": os.path.basename(a.out),
               "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE in separate passes; "
                         "bytes per launch averaged over all launches of the kernel", "kernels": {}}
        if "k_trace" in pmc:
            v = pmc["k_trace"]
            out["limiter"] = ("memory latency: waves wait on dependencies %.0f%% of their cycles (SQ_WAIT_ANY / "
                              "SQ_WAVE_CYCLES), VALU busy %.0f%%, L2 hit %.0f%%; HBM-side traffic well below peak"
                              % (100 * v.get("wait", 0), 100 * v.get("valu", 0), 100 * v.get("l2_hit", 0)))
            out["pmc"] = {k: pmc[k] for k in pmc if k in ("k_trace", "k_trace_packet", "k_shade")}
        for kn, v in traffic.items():
            f = v.get("FETCH_SIZE", (1, 0.0, 0))
            w = v.get("WRITE_SIZE", (1, 0.0, 0))
            out["kernels"][kn] = {"launches": f[0], "fetch_bytes": 2.0 * f[1] * 1024 / max(1, f[0]),
                                  "write_bytes": w[1] * 1024 / max(1, w[0])}
            out["kernels"][kn]["bytes_per_launch"] = out["kernels"][kn]["fetch_bytes"] + out["kernels"][kn]["write_bytes"]
        json.dump(out, open(a.json, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
