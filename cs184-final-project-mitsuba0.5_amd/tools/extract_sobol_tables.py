#!/usr/bin/env python3
"""Extract the Sobol (0,2)-sequence generator tables as binary data.

Provenance: the tables are the Joe & Kuo (2008) direction numbers
("new-joe-kuo-6.21201") expanded into generator matrices by L. Gruenschloss
(MIT licence, 2012).  The reference vendors them as C array literals in
``src/samplers/sobolseq.cpp`` (matrices32 at :33-53283, vdc_sobol_matrices at
:106537-107239, vdc_sobol_matrices_inv at :107241-107997).  This script reads
that file as *text*, parses the numeric literals and writes them as raw
little-endian arrays -- it never compiles or runs reference code.  The
reference sampler needs them for ``sobol::sampleSingle`` / ``sobol::look_up``
(``src/samplers/sobolseq.h:43-131``); our sampler restatement consumes the
same numbers.

Outputs (in ``data/sobol/``):
  matrices32.u32     1024 dims x 52 columns, uint32
  vdc.u64            R x 52, uint64   (vdc_sobol_matrices)
  vdc_inv.u64        R x 52, uint64   (vdc_sobol_matrices_inv)
  meta.json          row counts + sha256 of each file
Run once in a container that has /root/reference; the outputs are committed.
"""
import hashlib
import json
import os
import re
import sys

import numpy as np

SRC = "/root/reference/src/samplers/sobolseq.cpp"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "data", "sobol")

def parse_block(lines, start_pat):
    """Return all integer literals between the line holding start_pat and '};'."""
    i = next(k for k, l in enumerate(lines) if start_pat in l)
    vals = []
    for l in lines[i + 1:]:
        s = l.strip()
        if s.startswith("};"):
            break
        vals.extend(int(t.rstrip("ULul"), 0)
                    for t in re.findall(r"0x[0-9A-Fa-f]+[ULul]*|\b\d+[ULul]*\b", s))
    return vals


def main():
    if not os.path.exists(SRC):
        print("reference not present; tables are already committed", file=sys.stderr)
        return 1
    with open(SRC) as f:
        lines = f.readlines()
    os.makedirs(OUT, exist_ok=True)

    m32 = parse_block(lines, "Matrices::matrices32[")
    assert len(m32) == 1024 * 52, len(m32)
    a32 = np.array(m32, dtype=np.uint32)

    def table2d(pat):
        i = next(k for k, l in enumerate(lines) if pat in l)
        rows, cur, depth = [], [], 0
        for l in lines[i:]:
            s = l.split("//")[0].split("=")[-1].strip()
            if s.startswith("};"):
                break
            for tok in re.findall(r"\{|\}|0x[0-9A-Fa-f]+[ULul]*|\b\d+[ULul]*\b", s):
                if tok == "{":
                    depth += 1
                    if depth == 2:
                        cur = []
                elif tok == "}":
                    if depth == 2:
                        rows.append(cur + [0] * (52 - len(cur)))
                    depth -= 1
                else:
                    cur.append(int(tok.rstrip("ULul"), 0))
        return rows

    vdc = table2d("Matrices::vdc_sobol_matrices[]")
    vinv = table2d("Matrices::vdc_sobol_matrices_inv[]")
    assert all(len(r) == 52 for r in vdc) and all(len(r) == 52 for r in vinv)
    a_vdc = np.array(vdc, dtype=np.uint64)
    a_inv = np.array(vinv, dtype=np.uint64)

    meta = {"num_dimensions": 1024, "size": 52,
            "vdc_rows": int(a_vdc.shape[0]), "vdc_inv_rows": int(a_inv.shape[0]),
            "source": "src/samplers/sobolseq.cpp (Joe-Kuo 2008 / Gruenschloss 2012, MIT)"}
    for name, arr in (("matrices32.u32", a32), ("vdc.u64", a_vdc), ("vdc_inv.u64", a_inv)):
        b = arr.astype(arr.dtype.newbyteorder("<")).tobytes()
        with open(os.path.join(OUT, name), "wb") as f:
            f.write(b)
        meta[name] = hashlib.sha256(b).hexdigest()
    with open(os.path.join(OUT, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(json.dumps(meta, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
