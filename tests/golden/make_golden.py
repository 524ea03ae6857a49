#!/usr/bin/env python3
"""Generate golden vectors from the REFERENCE's own compilable pieces.

Builds oracle/ref.mk (drivers that include the reference headers
src/bsdfs/gausssexylingerie.hpp and src/bsdfs/InterpolatedDistribution1D.hpp
from /root/reference, outputs into oracle/_ref/) and records their outputs as
small JSON fixtures in tests/golden/.  Run in a container that has
/root/reference; the fixtures are committed and travel, the reference does not.
"""
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(HERE, "..", "..", "oracle")


def hexf(x):
    return float.hex(float(np.float32(x)))


def main():
    if not os.path.isdir("/root/reference"):
        print("no /root/reference here; fixtures are already committed")
        return 0
    subprocess.check_call(["make", "-s", "-f", "ref.mk"], cwd=ORACLE)

    # GaussLegendre<140> (marschner_diffuse.cpp:758)
    out = subprocess.check_output([os.path.join(ORACLE, "_ref", "gl140")], text=True)
    pts, wts = [], []
    for line in out.strip().splitlines():
        a, b = line.split()
        pts.append(a)
        wts.append(b)
    with open(os.path.join(HERE, "gl140.json"), "w") as f:
        json.dump({"source": "src/bsdfs/gausssexylingerie.hpp:11-93 (compiled by oracle/ref.mk)",
                   "points": pts, "weights": wts}, f, indent=0)

    # InterpolatedDistribution1D (marschner_diffuse.cpp:62, :68-77)
    rng = np.random.default_rng(1234)
    cases = []
    for case in range(3):
        size, ndist = (64, 64) if case < 2 else (16, 5)
        w = rng.random((ndist, size)).astype(np.float32) ** 3
        if case == 1:
            w[5, :] = 1e-7  # degenerate row -> uniform fallback (:51-58)
            w[:, 10:20] = 0.0
        n = 400
        dist = np.concatenate([rng.uniform(-1.0, ndist + 1.0, n - 8),
                               [0.0, ndist - 1.0, ndist - 1 + 0.999, 5.0, 5.5, 4.5, 0.25, 63.0]]).astype(np.float32)
        u = np.concatenate([rng.random(n - 8), [0.0, 1.0, 0.5, 0.999999, 0.3, 1e-7, 0.9, 0.0]]).astype(np.float32)
        inp = [f"{size} {ndist} {n}"]
        inp += [float.hex(float(v)) for v in w.reshape(-1)]
        inp += [f"{float.hex(float(d))} {float.hex(float(x))}" for d, x in zip(dist, u)]
        res = subprocess.run([os.path.join(ORACLE, "_ref", "idist")], input="\n".join(inp) + "\n",
                             text=True, capture_output=True, check=True).stdout
        rows = [l.split() for l in res.strip().splitlines()]
        cases.append({"size": size, "ndist": ndist,
                      "weights": [float.hex(float(v)) for v in w.reshape(-1)],
                      "dist": [float.hex(float(v)) for v in dist],
                      "u": [float.hex(float(v)) for v in u],
                      "out_x": [int(r[0]) for r in rows],
                      "out_u": [r[1] for r in rows], "out_pdf": [r[2] for r in rows],
                      "out_sum": [r[3] for r in rows]})
    with open(os.path.join(HERE, "idist.json"), "w") as f:
        json.dump({"source": "src/bsdfs/InterpolatedDistribution1D.hpp:7-111 (compiled by oracle/ref.mk)",
                   "cases": cases}, f)
    print("golden fixtures written")
    return 0


if __name__ == "__main__":
    sys.exit(main())
