#!/usr/bin/env python3
"""Summarise the FETCH_SIZE / WRITE_SIZE calibration (tools/fetch_calib.hip under
rocprofv3 --pmc, scripts/archive/r03_fetch_calib.sh): per launch, the counter in bytes
divided by the lines the launch touched and by the bytes it requested.

Usage: python tools/fetch_calib.py <dir with fetch/ and write/ rocpd outputs> <program stdout>
"""
import glob
import json
import os
import sqlite3
import sys


def per_dispatch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    if not f:
        raise SystemExit("no rocpd db under %s" % d)
    db = sqlite3.connect(f[0])
    cur = db.execute("select * from counters_collection")
    cols = [c[0] for c in cur.description]
    rows = [dict(zip(cols, r)) for r in cur.fetchall()]
    key = next(k for k in ("dispatch_id", "dispatch", "id") if k in cols)
    vals = {}
    for r in rows:  # the program's own kernels only (not the runtime's fill kernel)
        name = str(r.get("kernel_name", ""))
        if r.get("counter_name") == counter and ("k_gather" in name or "k_stream" in name or "k_scatter" in name):
            vals[r[key]] = vals.get(r[key], 0.0) + float(r["value"])
    return [vals[k] for k in sorted(vals)]


def main():
    d, log = sys.argv[1], sys.argv[2]
    launches = []
    for line in open(log):
        if line.startswith("launch "):
            t = line.split()
            launches.append({"name": t[2], "lines": int(t[4]), "record": int(t[6])})
    fetch = per_dispatch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "write"), "WRITE_SIZE")
    out = []
    for i, l in enumerate(launches):
        is_write = l["name"] in ("stream_write", "scatter16")
        v = (write if is_write else fetch)[i] * 1024.0  # the counters are in KiB
        req = l["lines"] * l["record"]
        out.append({"launch": l["name"], "counter": "WRITE_SIZE" if is_write else "FETCH_SIZE",
                    "counter_bytes": v, "requested_bytes": req, "lines": l["lines"],
                    "counter_bytes_per_line": round(v / l["lines"], 2),
                    "counter_over_requested": round(v / req, 4)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
