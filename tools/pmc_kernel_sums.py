"""Per-kernel counter sums from a rocprofv3 --pmc run (rocpd database): one line per kernel.
Usage: python tools/pmc_kernel_sums.py <dir with the .db> [kernel-substring ...]"""
import glob
import os
import sqlite3
import sys

d = sys.argv[1]
want = sys.argv[2:]
db = sqlite3.connect(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0])
rows = {}
for kn, ctr, val, n in db.execute("select kernel_name, counter_name, sum(value), count(*) from counters_collection "
                                  "group by kernel_name, counter_name"):
    if want and not any(w == kn or w in kn for w in want):
        continue
    rows.setdefault(kn, {})[ctr] = (val, n)
for kn, c in sorted(rows.items()):
    print(kn, " ".join("%s=%.4g" % (k, v[0]) for k, v in sorted(c.items())), "launches=%d" % next(iter(c.values()))[1])
