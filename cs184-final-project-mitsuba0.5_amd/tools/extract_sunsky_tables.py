#!/usr/bin/env python3
"""Extract the numeric tables the sunsky emitter needs from the reference's
sources into data files (data only; no code is copied):

  src/emitters/sunsky/skymodeldata.h  datasetRGB{1,2,3} (1080 doubles each) and
                                      datasetRGBRad{1,2,3} (120 doubles each):
                                      the Hosek-Wilkie RGB sky model coefficients
  src/libcore/spectrum.cpp            CIE 1931 wavelengths and x/y/z matching
                                      functions (471 floats each)
  src/emitters/sunsky/sunmodel.h      Preetham sun attenuation tables
                                      (k_o, k_g, k_wa, solar amplitude)

Outputs (data/sunsky/): hosek_rgb.f64 (3x1080 then 3x120 doubles, little
endian), cie1931.f32 (wavelengths, x, y, z; 4x471 floats), sun_tables.json
(float32-rounded values), meta.json (sha256 of every output).
Usage: extract_sunsky_tables.py /root/reference <out_dir>
"""
import hashlib
import json
import os
import re
import sys

import numpy as np


def strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def array(src, name):
    m = re.search(r"\b%s\s*\[[^\]]*\]\s*=\s*\{(.*?)\}" % re.escape(name), src, flags=re.S)
    if not m:
        raise SystemExit("array %s not found" % name)
    return [float(t) for t in re.split(r"[,\s]+", m.group(1).strip()) if t]


def main():
    ref, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    sky = strip_comments(open(os.path.join(ref, "src/emitters/sunsky/skymodeldata.h")).read())
    rgb = [array(sky, "datasetRGB%d" % i) for i in (1, 2, 3)]
    rad = [array(sky, "datasetRGBRad%d" % i) for i in (1, 2, 3)]
    assert all(len(a) == 1080 for a in rgb) and all(len(a) == 120 for a in rad)
    np.array(rgb + rad, dtype=object)  # shape check only
    np.concatenate([np.array(a, "<f8") for a in rgb + rad]).tofile(os.path.join(out, "hosek_rgb.f64"))

    spec = strip_comments(open(os.path.join(ref, "src/libcore/spectrum.cpp")).read())
    cie = [array(spec, n) for n in ("CIE_wavelengths", "CIE_X_entries", "CIE_Y_entries", "CIE_Z_entries")]
    assert all(len(a) == 471 for a in cie)
    np.concatenate([np.array(a, "<f4") for a in cie]).tofile(os.path.join(out, "cie1931.f32"))

    sun = strip_comments(open(os.path.join(ref, "src/emitters/sunsky/sunmodel.h")).read())
    tabs = {}
    for n in ("k_oWavelengths", "k_oAmplitudes", "k_gWavelengths", "k_gAmplitudes", "k_waWavelengths",
              "k_waAmplitudes", "solWavelengths", "solAmplitudes"):
        tabs[n] = [float(np.float32(v)) for v in array(sun, n)]
    json.dump(tabs, open(os.path.join(out, "sun_tables.json"), "w"), indent=0)

    meta = {}
    for f in ("hosek_rgb.f64", "cie1931.f32", "sun_tables.json"):
        meta[f] = hashlib.sha256(open(os.path.join(out, f), "rb").read()).hexdigest()
    json.dump(meta, open(os.path.join(out, "meta.json"), "w"), indent=1)
    print({k: len(v) for k, v in tabs.items()}, "ok")


if __name__ == "__main__":
    main()
