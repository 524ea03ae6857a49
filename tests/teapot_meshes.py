"""Substitute meshes for the C1 "teapot" plumbing scene (BASELINE.json configs[0]).

models/teapot/scene.xml:56-72 loads models/Mesh001.obj and models/Mesh000.obj,
which the reference repository does not ship.  This module writes two seeded
stand-ins of teapot scale (the scene's camera frames about 16 units at the
origin; the floor rectangle lies in y = 0):

  Mesh001.obj  a bumpy body, UV sphere r ~ 3.3 on the floor, 96 x 48 segments,
               with per-vertex normals and texture coordinates, faces
               "v/vt/vn", poles as triangle fans (~9k triangles)
  Mesh000.obj  two groups: "handle", a torus WITHOUT normals or texture
               coordinates (smooth normals are computed, trimesh.cpp:608-681)
               written as quads with a mix of positive and negative indices
               (fan triangulation, obj.cpp:309-323, 640-645); "knob", a small
               sphere on top with faces "v//vn"

They exercise every OBJ face form and mesh path of obj.cpp / trimesh.cpp the
scene reaches.  Deterministic for a given seed (numpy default_rng).
"""
import os

import numpy as np


def _fmt(a):
    return " ".join("%.6f" % x for x in a)


def _sphere(center, radius, nu, nv, rng, bump):
    """vertices (ring-major, poles separate), normals, uv; rings exclude the poles"""
    verts, norms, uvs = [], [], []
    for j in range(1, nv):
        theta = np.pi * j / nv
        for i in range(nu):
            phi = 2 * np.pi * i / nu
            n = np.array([np.sin(theta) * np.cos(phi), np.cos(theta), np.sin(theta) * np.sin(phi)])
            r = radius * (1.0 + bump * rng.uniform(-1, 1))
            verts.append(center + r * n)
            norms.append(n)
            uvs.append((i / nu, j / nv))
    top = center + np.array([0, radius, 0])
    bot = center - np.array([0, radius, 0])
    return np.array(verts), np.array(norms), np.array(uvs), top, bot


def write_body(path, seed=2024):
    rng = np.random.default_rng(seed)
    nu, nv, R = 96, 48, 3.3
    c = np.array([0.0, R, 0.0])
    V, N, UV, top, bot = _sphere(c, R, nu, nv, rng, 0.01)
    lines = ["# C1 substitute body (tests/teapot_meshes.py, seed %d)" % seed]
    lines += ["v " + _fmt(v) for v in V]
    lines += ["v " + _fmt(top), "v " + _fmt(bot)]
    lines += ["vn " + _fmt(n) for n in N]
    lines += ["vn 0 1 0", "vn 0 -1 0"]
    lines += ["vt %.6f %.6f" % tuple(t) for t in UV]
    lines += ["vt 0.5 0", "vt 0.5 1"]
    nring = V.shape[0]
    itop, ibot = nring + 1, nring + 2  # 1-based
    vid = lambda j, i: (j * nu + (i % nu)) + 1  # ring j in [0, nv-2]
    f = lambda a: "%d/%d/%d" % (a, a, a)
    for j in range(nv - 2):
        for i in range(nu):
            a, b, cc, d = vid(j, i), vid(j, i + 1), vid(j + 1, i + 1), vid(j + 1, i)
            lines.append("f %s %s %s %s" % (f(a), f(d), f(cc), f(b)))  # quad -> fan of two
    for i in range(nu):
        lines.append("f %s %s %s" % (f(itop), f(vid(0, i)), f(vid(0, i + 1))))
        lines.append("f %s %s %s" % (f(ibot), f(vid(nv - 2, i + 1)), f(vid(nv - 2, i))))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def write_handle_and_knob(path, seed=2025):
    rng = np.random.default_rng(seed)
    lines = ["# C1 substitute handle + knob (tests/teapot_meshes.py, seed %d)" % seed, "g handle"]
    # torus in the yz plane behind the body (the camera looks along about -x)
    nu, nv, Rmaj, rmin = 48, 16, 1.6, 0.35
    cen = np.array([0.0, 3.6, -3.6])
    V = []
    for i in range(nu):
        a = 2 * np.pi * i / nu
        ring = np.array([0.0, np.cos(a), np.sin(a)])
        for j in range(nv):
            b = 2 * np.pi * j / nv
            r = rmin * (1.0 + 0.02 * rng.uniform(-1, 1))
            p = cen + Rmaj * ring + r * (np.cos(b) * ring + np.sin(b) * np.array([1.0, 0, 0]))
            V.append(p)
    lines += ["v " + _fmt(v) for v in V]
    nvert = len(V)
    for i in range(nu):
        for j in range(nv):
            ids = [((i % nu) * nv + j % nv), (((i + 1) % nu) * nv + j % nv),
                   (((i + 1) % nu) * nv + (j + 1) % nv), ((i % nu) * nv + (j + 1) % nv)]
            if (i + j) % 2:  # negative (relative) indices: -1 is the last vertex written so far
                lines.append("f " + " ".join(str(k - nvert) for k in ids))
            else:
                lines.append("f " + " ".join(str(k + 1) for k in ids))
    # knob: a small sphere on top of the body, faces v//vn
    lines.append("g knob")
    base = nvert
    kn, kv, kr = 24, 12, 0.45
    kc = np.array([0.0, 6.6 + kr * 0.8, 0.0])
    Vk, Nk, _, top, bot = _sphere(kc, kr, kn, kv, rng, 0.0)
    lines += ["v " + _fmt(v) for v in Vk]
    lines += ["v " + _fmt(top), "v " + _fmt(bot)]
    lines += ["vn " + _fmt(n) for n in Nk]
    lines += ["vn 0 1 0", "vn 0 -1 0"]
    nr = Vk.shape[0]
    vid = lambda j, i: (j * kn + (i % kn))
    f = lambda k: "%d//%d" % (base + k + 1, k + 1)
    for j in range(kv - 2):
        for i in range(kn):
            lines.append("f %s %s %s" % (f(vid(j, i)), f(vid(j + 1, i)), f(vid(j + 1, i + 1))))
            lines.append("f %s %s %s" % (f(vid(j, i)), f(vid(j + 1, i + 1)), f(vid(j, i + 1))))
    for i in range(kn):
        lines.append("f %s %s %s" % (f(nr), f(vid(0, i)), f(vid(0, i + 1))))
        lines.append("f %s %s %s" % (f(nr + 1), f(vid(kv - 2, i + 1)), f(vid(kv - 2, i))))
    with open(path, "w") as fh:
        fh.write("\n".join(lines) + "\n")


def write_all(models_dir):
    os.makedirs(models_dir, exist_ok=True)
    write_body(os.path.join(models_dir, "Mesh001.obj"))
    write_handle_and_knob(os.path.join(models_dir, "Mesh000.obj"))


if __name__ == "__main__":
    import sys

    write_all(sys.argv[1] if len(sys.argv) > 1 else "models")
