#!/usr/bin/env python3
"""Extract the ldrfilm banner mask from the reference's sources (data only):

  src/films/banner.h   bannerWidth x bannerHeight chars; 0 marks a pixel the
                       banner paints white (ldrfilm.cpp:323-332)

Output: data/film/banner.u8 (row-major bytes), data/film/banner.json
({"width", "height", "sha256"}).
Usage: extract_banner.py /root/reference <out_dir>
"""
import hashlib
import json
import os
import re
import sys


def main():
    ref, out = sys.argv[1], sys.argv[2]
    src = open(os.path.join(ref, "src/films/banner.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    w = int(re.search(r"bannerWidth\s*=\s*(\d+)", src).group(1))
    h = int(re.search(r"bannerHeight\s*=\s*(\d+)", src).group(1))
    body = re.search(r"banner\s*\[\s*\]\s*=\s*\{(.*?)\}", src, flags=re.S).group(1)
    vals = bytes(int(t) for t in re.split(r"[,\s]+", body.strip()) if t)
    if len(vals) != w * h:
        raise SystemExit("banner size mismatch: %d != %d x %d" % (len(vals), w, h))
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "banner.u8"), "wb") as f:
        f.write(vals)
    with open(os.path.join(out, "banner.json"), "w") as f:
        json.dump({"width": w, "height": h, "sha256": hashlib.sha256(vals).hexdigest()}, f, indent=1)


if __name__ == "__main__":
    main()
