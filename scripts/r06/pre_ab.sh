#!/bin/bash
# A/B on one box: the per-record pre-test radius classes vs one global radius (libv_glob), main twice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/cs184-final-project-mitsuba0.5_amd
run() { # name lib
  HAIRPT_LIB=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/ab_$1.json 2> $O/ab_$1.err || return $?
  python3 - $1 <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/r06/ab_%s.json" % v).read().strip().splitlines()[-1])
print(v, d["value"], d["ms_per_step"], d["roofline"].get("rank0_trace_ms_per_step"), d["stats"]["exact_tests_per_ray"], d["stats"].get("film_fingerprint"))
PY
}
run main1 $L/lib/libhairpt.so && run glob $L/libv_glob/libhairpt.so && run main2 $L/lib/libhairpt.so && run glob2 $L/libv_glob/libhairpt.so
