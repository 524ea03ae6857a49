#!/bin/bash
# k_trace pre-test variants: parity tests,
# then bench A/B against the previous build (libv_prev), alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py::test_folded_strands_match_oracle_and_keep_the_pretest -m gpu -x -q --timeout 300 --timeout-method thread > $O/ur_tests.log 2>&1; rc=$?; tail -1 $O/ur_tests.log; [ $rc -eq 0 ] || exit $rc
L=$PWD/cs184-final-project-mitsuba0.5_amd
run() { # name lib
  HAIRPT_LIB=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/ur_$1.json 2> $O/ur_$1.err || return $?
  python3 - $1 <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/r06/ur_%s.json" % v).read().strip().splitlines()[-1])
k = d["roofline"].get("kernel_ms_per_step") or d.get("kernel_ms_per_step") or {}
def find(o, key):
    if isinstance(o, dict):
        for kk, x in o.items():
            if kk == key: return x
            r = find(x, key)
            if r is not None: return r
k = find(d, "kernel_ms_per_step") or {}
print(v, d["value"], d["ms_per_step"], d["stats"]["exact_tests_per_ray"], d["stats"].get("film_fingerprint"), {x: k.get(x) for x in ("trace_packet", "trace", "tail")})
PY
}
run main $L/lib/libhairpt.so && run prev $L/libv_prev/libhairpt.so && run main2 $L/lib/libhairpt.so && run prev2 $L/libv_prev/libhairpt.so
