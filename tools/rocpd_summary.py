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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir", help="gpurun_out/prof_<tag> (trace/, fetch/, write/)")
    ap.add_argument("--out", required=True)
    ap.add_argument("--title", default="")
    ap.add_argument("--json", default=None, help="also write per-launch traffic as JSON (read by bench.py)")
    ap.add_argument("--workload", default="", help="workload string the traffic belongs to (bench config)")
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
    open(a.out, "w").write("\n".join(lines) + "\n")
    if a.json:
        import json

        out = {"workload": a.workload, "source": os.path.basename(a.out),
               "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE in separate passes; "
                         "bytes per launch averaged over all launches of the kernel", "kernels": {}}
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
