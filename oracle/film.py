"""Film development restated in numpy -- TEST INFRASTRUCTURE ONLY.

The checker for the product's host-side film code (csrc/host/film.cpp,
hpt_write_film): only tests/ use it.  Parity unpinned against the reference
binary (the films need Boost / libpng / OpenEXR); follows, in float32:

  ImageBlock -> RGB          src/libcore/fmtconv.cpp:956-990  (spec * (1/weight))
  gamma / sRGB, 8-bit        src/libcore/fmtconv.cpp:1093-1160
  Reinhard tonemapping       src/libcore/bitmap.cpp:1711-1852
  exposure multiplier        src/films/ldrfilm.cpp:300-321
  banner                     src/films/ldrfilm.cpp:323-332, hdrfilm.cpp:492-502
plus minimal readers for the PNG / PFM / RGBE / OpenEXR files the product writes.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

f32 = np.float32


def resolve(film_rgbw, luminance=False):
    """(H, W, 4) accumulated film -> (H, W, C) float32 like the weighted-RGBA converter."""
    film = np.asarray(film_rgbw, np.float32)
    w = film[..., 3]
    inv = np.where(w != 0, f32(1) / np.where(w != 0, w, f32(1)), w).astype(np.float32)
    if luminance:
        lum = (film[..., 0] * f32(0.212671) + film[..., 1] * f32(0.715160)) + film[..., 2] * f32(0.072169)
        return (lum * inv)[..., None].astype(np.float32)
    return (film[..., :3] * inv[..., None]).astype(np.float32)


def apply_gamma(v, inv_gamma):
    v = v.astype(np.float32)
    if inv_gamma == -1:
        with np.errstate(invalid="ignore"):
            hi = f32(1.055) * np.power(v, f32(1.0 / 2.4)) - f32(0.055)
        return np.where(v <= f32(0.0031308), f32(12.92) * v, hi).astype(np.float32)
    with np.errstate(invalid="ignore"):
        return np.power(v, f32(inv_gamma)).astype(np.float32)


def to_u8(v, multiplier=1.0, inv_gamma=-1.0):
    v = v.astype(np.float32) * f32(multiplier)
    if inv_gamma != 1:
        v = apply_gamma(v, inv_gamma)
    x = v * f32(255) + f32(0.5)
    x = np.where(np.isnan(x), f32(0), x)  # std::max(0, NaN) == 0
    return np.minimum(f32(255), np.maximum(f32(0), x)).astype(np.uint8)


def reinhard(px, key=0.18, burn=0.0):
    px = px.astype(np.float32).copy()
    C = px.shape[-1]
    flat = px.reshape(-1, C)
    lum = (flat[:, 0] * f32(0.212671) + flat[:, 1] * f32(0.715160) + flat[:, 2] * f32(0.072169)) if C == 3 \
        else flat[:, 0]
    # the max luminance is reset by a pixel of exactly 1024 (the HDR banner)
    maxl = f32(0)
    last = np.nonzero(lum == 1024)[0]
    start = last[-1] if last.size else 0
    maxl = f32(lum[start:].max()) if lum.size else f32(0)
    acc = f32(0)
    for v in lum:  # float32 running sum, like the reference loop
        acc = f32(acc + f32(np.log(np.float64(f32(1e-3) + v))))
    logavg = f32(np.exp(np.float64(acc / f32(lum.size))))
    if maxl == 0:
        return px
    burn = min(f32(1), max(f32(1e-8), f32(1) - f32(burn)))
    scale = f32(key) / logavg
    lwhite = maxl * scale
    inv_wp2 = f32(1) / (lwhite * lwhite * f32(np.power(burn, f32(4))))
    if C == 1:
        lp = flat[:, 0] * scale
        flat[:, 0] = lp * (f32(1) + lp * inv_wp2) / (f32(1) + lp)
        return px
    r, g, b = flat[:, 0], flat[:, 1], flat[:, 2]
    X = r * f32(0.412453) + g * f32(0.357580) + b * f32(0.180423)
    Y = r * f32(0.212671) + g * f32(0.715160) + b * f32(0.072169)
    Z = r * f32(0.019334) + g * f32(0.119193) + b * f32(0.950227)
    norm = f32(1) / (X + Y + Z)
    x, y, lp = X * norm, Y * norm, Y * scale
    Y = lp * (f32(1) + lp * inv_wp2) / (f32(1) + lp)
    ratio = Y / y
    X = ratio * x
    Z = ratio * (f32(1) - x - y)
    flat[:, 0] = f32(3.240479) * X + f32(-1.537150) * Y + f32(-0.498535) * Z
    flat[:, 1] = f32(-0.969256) * X + f32(1.875991) * Y + f32(0.041556) * Z
    flat[:, 2] = f32(0.055648) * X + f32(-0.204043) * Y + f32(1.057311) * Z
    return px


def banner_mask(mask_bytes, w, h, bw=108, bh=5):
    """(H, W) bool: pixels the banner paints (mask value 0) when it fits."""
    out = np.zeros((h, w), bool)
    if w > bw + 5 and h > bh + 5:
        m = np.frombuffer(mask_bytes, np.uint8).reshape(bh, bw) == 0
        out[h - bh - 5:h - 5, w - bw - 5:w - 5] = m
    return out


def develop_ldr(film_rgbw, gamma=-1.0, exposure=0.0, reinhard_tm=False, key=0.18, burn=0.0, luminance=False,
                banner=None):
    px = resolve(film_rgbw, luminance)
    mult = 1.0
    if reinhard_tm:
        px = reinhard(px, key, burn)
    else:
        mult = f32(np.power(f32(2), f32(exposure)))
    inv = -1.0 if gamma == -1 else float(f32(1) / f32(gamma))
    out = to_u8(px, mult, inv)
    if banner is not None:
        out[banner] = 255
    return out


# ---- readers -------------------------------------------------------------
def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        t = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert zlib.crc32(t + body) & 0xffffffff == crc
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", body[:10])
            ch = {0: 1, 4: 2, 2: 3, 6: 4}[ctype]
        elif t == b"IDAT":
            idat += body
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * ch)
    assert np.all(raw[:, 0] == 0)
    return raw[:, 1:].reshape(h, w, ch)


def read_pfm(path):
    data = open(path, "rb").read()
    parts = data.split(b"\n", 3)
    ch = 3 if parts[0] == b"PF" else 1
    w, h = map(int, parts[1].split())
    assert float(parts[2]) < 0
    img = np.frombuffer(parts[3], "<f4").reshape(h, w, ch)
    return img[::-1]


def read_rgbe(path):
    data = open(path, "rb").read()
    end = data.index(b"\n-Y ")
    header_end = data.index(b"\n", end + 1)
    _, h, _, w = data[end + 1:header_end].split()
    h, w = int(h), int(w)
    pos = header_end + 1
    out = np.zeros((h, w, 4), np.uint8)
    for y in range(h):
        assert data[pos:pos + 2] == b"\x02\x02"
        pos += 4
        for c in range(4):
            x = 0
            while x < w:
                n = data[pos]
                pos += 1
                if n > 128:
                    out[y, x:x + n - 128, c] = data[pos]
                    pos += 1
                    x += n - 128
                else:
                    out[y, x:x + n, c] = np.frombuffer(data[pos:pos + n], np.uint8)
                    pos += n
                    x += n
    e = out[..., 3].astype(np.int32)
    f = np.where(e > 0, np.ldexp(np.float32(1), e - (128 + 8)), 0).astype(np.float32)
    return out[..., :3].astype(np.float32) * f[..., None], out


def rgbe_encode(px):
    """RGBE_FromFloat (bitmap.cpp:3504-3520) in numpy."""
    mx = px.max(axis=-1)
    m, e = np.frexp(mx)
    scale = np.where(mx < 1e-32, 0, (m.astype(np.float32) * f32(256)) / np.where(mx < 1e-32, 1, mx)).astype(np.float32)
    rgb = (px * scale[..., None]).astype(np.float32)
    out = np.zeros(px.shape[:-1] + (4,), np.uint8)
    out[..., :3] = np.where(mx[..., None] < 1e-32, 0, np.trunc(rgb)).astype(np.uint8)
    out[..., 3] = np.where(mx < 1e-32, 0, e + 128).astype(np.uint8)
    return out


def read_exr(path):
    data = open(path, "rb").read()
    assert data[:4] == b"\x76\x2f\x31\x01"
    pos = 8
    chans, box = [], None
    while data[pos] != 0:
        name_end = data.index(b"\0", pos)
        name = data[pos:name_end].decode()
        type_end = data.index(b"\0", name_end + 1)
        size, = struct.unpack("<i", data[type_end + 1:type_end + 5])
        val = data[type_end + 5:type_end + 5 + size]
        if name == "channels":
            p = 0
            while val[p] != 0:
                e = val.index(b"\0", p)
                cname = val[p:e].decode()
                ptype, = struct.unpack("<i", val[e + 1:e + 5])
                chans.append((cname, ptype))
                p = e + 17
        elif name == "dataWindow":
            box = struct.unpack("<4i", val)
        elif name == "compression":
            assert val[0] == 0
        pos = type_end + 5 + size
    pos += 1
    w, h = box[2] - box[0] + 1, box[3] - box[1] + 1
    offsets = struct.unpack("<%dQ" % h, data[pos:pos + 8 * h])
    dt = {1: "<f2", 2: "<f4", 0: "<u4"}
    out = {c: np.zeros((h, w), np.float32 if t else np.uint32) for c, t in chans}
    for yy, off in enumerate(offsets):
        y, n = struct.unpack("<ii", data[off:off + 8])
        p = off + 8
        for c, t in chans:
            nb = w * (2 if t == 1 else 4)
            out[c][y] = np.frombuffer(data[p:p + nb], dt[t])
            p += nb
    return out
