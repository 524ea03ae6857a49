"""Synthetic hair geometry in the reference's BINARY_HAIR format.

The reference's models/*/models/*.mitshair blobs are not shipped
(.MISSING_LARGE_BLOBS), so every config renders deterministic synthetic
strands placed where the scene cameras look.
Format (src/shapes/hair.cpp:92-98, :656-716): b"BINARY_HAIR", uint32 vertex
count, then float32 xyz; a +inf float precedes the first vertex of each
strand.  Consecutive segments turn by more than the loader's 1 degree merge
threshold (hair.cpp:615-616), so no vertex is merged away.
"""
from __future__ import annotations

import math
import os
import struct

import numpy as np


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def _perp(d, rng):
    a = rng.normal(size=d.shape)
    a -= (a * d).sum(-1, keepdims=True) * d
    return _unit(a)


def _rotate(d, axis, ang):
    """Rodrigues rotation of unit vectors d about unit axes by angles (radians)."""
    c = np.cos(ang)[:, None]
    s = np.sin(ang)[:, None]
    return d * c + np.cross(axis, d) * s + axis * (axis * d).sum(-1, keepdims=True) * (1 - c)


def _strands(roots, dirs, nseg, seglen, turn_deg, rng, gravity=0.0):
    """Grow strands by rotating the tangent 'turn_deg' degrees per segment; (N, nseg+1, 3)."""
    n = roots.shape[0]
    pts = np.empty((n, nseg + 1, 3), dtype=np.float64)
    pts[:, 0] = roots
    d = dirs.copy()
    axis = _perp(d, rng)
    for k in range(nseg):
        ang = np.deg2rad(rng.uniform(turn_deg[0], turn_deg[1], size=n))
        axis = _unit(axis + 0.3 * _perp(d, rng))
        axis = _unit(axis - (axis * d).sum(-1, keepdims=True) * d)
        d = _rotate(d, axis, ang)
        if gravity:
            d = _unit(d + np.array([0.0, -gravity, 0.0]))
        pts[:, k + 1] = pts[:, k] + d * seglen[:, None]
    return pts


def furball(n_strands: int, seed: int = 1):
    """Sphere of radius 2.3 at (0, 12.3, 0), 6-10 segments per strand (models/furball)."""
    rng = np.random.default_rng(seed)
    centre = np.array([0.0, 12.3, 0.0])
    nrm = _unit(rng.normal(size=(n_strands, 3)))
    roots = centre + 2.3 * nrm
    out = []
    nseg_all = rng.integers(6, 11, size=n_strands)
    for nseg in range(6, 11):
        idx = np.nonzero(nseg_all == nseg)[0]
        if idx.size == 0:
            continue
        seglen = rng.uniform(0.12, 0.25, size=idx.size)
        dirs = _unit(nrm[idx] + 0.25 * rng.normal(size=(idx.size, 3)))
        out.extend(_strands(roots[idx], dirs, nseg, seglen, (2.0, 10.0), rng, gravity=0.02))
    return out


def straight(n_strands: int, nseg: int = 24, seed: int = 2):
    """Scalp cap centred at (0, 14, 0), strands falling along -y to y~4 (models/straight-hair)."""
    rng = np.random.default_rng(seed)
    centre = np.array([0.0, 14.0, 0.0])
    u = rng.uniform(0.0, 1.0, size=n_strands)
    theta = np.arccos(1 - 0.9 * u)  # upper cap
    phi = rng.uniform(0, 2 * math.pi, size=n_strands)
    nrm = np.stack([np.sin(theta) * np.cos(phi), np.cos(theta), np.sin(theta) * np.sin(phi)], -1)
    roots = centre + 4.5 * nrm
    dirs = _unit(nrm * 0.4 + np.array([0.0, -1.0, 0.0]) + 0.05 * rng.normal(size=(n_strands, 3)))
    length = np.clip(roots[:, 1] - 4.0, 2.0, None)
    seglen = length / nseg
    return list(_strands(roots, dirs, nseg, seglen, (1.5, 4.0), rng, gravity=0.15))


def curly(n_strands: int, nseg: int = 270, seed: int = 3):
    """Helical strands hanging from the straight-hair cap (models/curly-hair)."""
    rng = np.random.default_rng(seed)
    centre = np.array([0.0, 14.0, 0.0])
    u = rng.uniform(0.0, 1.0, size=n_strands)
    theta = np.arccos(1 - 0.9 * u)
    phi = rng.uniform(0, 2 * math.pi, size=n_strands)
    nrm = np.stack([np.sin(theta) * np.cos(phi), np.cos(theta), np.sin(theta) * np.sin(phi)], -1)
    roots = centre + 4.6 * nrm
    radius = rng.uniform(0.2, 0.4, size=n_strands)
    pitch = rng.uniform(0.3, 0.6)
    phase = rng.uniform(0, 2 * math.pi, size=n_strands)
    up = np.array([0.0, 1.0, 0.0])
    pts = np.empty((n_strands, nseg + 1, 3))
    u0 = np.array([1.0, 0.0, 0.0])
    w0 = np.array([0.0, 0.0, 1.0])
    for k in range(nseg + 1):
        ang = phase + k * 2 * math.pi / 12.0
        drop = (pitch / 12.0) * k * (1.0 + 0.3 * np.sin(phase))
        c = roots - up[None, :] * drop[:, None] if np.ndim(drop) else roots - up * drop
        pts[:, k] = c + radius[:, None] * (np.cos(ang)[:, None] * u0 + np.sin(ang)[:, None] * w0)
    return list(pts)


def curl_lock(n_strands: int, lock: int, nseg: int = 60, seed: int = 4):
    """One of the four hanging curly locks of models/hair-curl (black, red,
    brown, blonde; the camera at z = 17 looks down -z at y ~ 5.9): lock k
    hangs at x = -3.6 + 2.4 k from y ~ 9.5 down to y ~ 2.5, helical curls of
    radius 0.08-0.2 around a slightly swaying axis."""
    rng = np.random.default_rng(seed * 16 + lock)
    cx = -3.6 + 2.4 * lock
    roots = np.stack([cx + rng.uniform(-0.7, 0.7, n_strands), 9.5 + rng.uniform(-0.15, 0.15, n_strands),
                      rng.uniform(-0.5, 0.5, n_strands)], -1)
    radius = rng.uniform(0.08, 0.2, size=n_strands)
    turns = rng.uniform(5.0, 9.0, size=n_strands)
    length = rng.uniform(5.5, 7.0, size=n_strands)
    phase = rng.uniform(0, 2 * math.pi, size=n_strands)
    sway = rng.uniform(-0.3, 0.3, size=(n_strands, 2))
    k = np.arange(nseg + 1)[None, :] / nseg
    ang = phase[:, None] + 2 * math.pi * turns[:, None] * k
    pts = np.empty((n_strands, nseg + 1, 3))
    pts[..., 0] = roots[:, 0:1] + sway[:, 0:1] * k ** 2 + radius[:, None] * np.cos(ang)
    pts[..., 1] = roots[:, 1:2] - length[:, None] * k
    pts[..., 2] = roots[:, 2:3] + sway[:, 1:2] * k ** 2 + radius[:, None] * np.sin(ang)
    return list(pts)


def write_binary_hair(path: str, strands) -> int:
    """Write strands (iterable of (n_i, 3) arrays) as BINARY_HAIR; returns vertex count."""
    nvert = sum(len(s) for s in strands)
    chunks = []
    inf = np.array([np.inf], dtype="<f4")
    for s in strands:
        chunks.append(inf)
        chunks.append(np.asarray(s, dtype="<f4").reshape(-1))
    body = np.concatenate(chunks) if chunks else np.zeros(0, dtype="<f4")
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "wb") as f:
        f.write(b"BINARY_HAIR")
        f.write(struct.pack("<I", nvert))
        f.write(body.astype("<f4").tobytes())
    return nvert


def write_ascii_hair(path: str, strands) -> int:
    nvert = 0
    with open(path, "w") as f:
        for i, s in enumerate(strands):
            if i:
                f.write("\n")
            for p in np.asarray(s, dtype=np.float32):
                f.write("%.9g %.9g %.9g\n" % (float(p[0]), float(p[1]), float(p[2])))
                nvert += 1
    return nvert
