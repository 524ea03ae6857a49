#!/bin/bash
# per-leaf pre-test radius, unconditional load: bench A/B against libv_base, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
L=$PWD/cs184-final-project-mitsuba0.5_amd
run() { # name lib
  HAIRPT_LIB=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/lr_$1.json 2> $O/lr_$1.err || return $?
  python3 - $1 <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/r06/lr_%s.json" % v).read().strip().splitlines()[-1])
def find(o, key):
    if isinstance(o, dict):
        for k, x in o.items():
            if k == key: return x
            r = find(x, key)
            if r is not None: return r
k = find(d, "kernel_ms_per_step") or {}
print(v, d["value"], d["ms_per_step"], d["stats"]["exact_tests_per_ray"], d["stats"].get("film_fingerprint"),
      {x: k.get(x) for x in ("camera", "trace_packet", "primary", "trace")})
PY
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_camera.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/lr_tests.log 2>&1; rc=$?; grep -E "passed|failed|Error|folded|fold-free" $O/lr_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
run main $L/lib/libhairpt.so && run base $L/libv_base/libhairpt.so && run main2 $L/lib/libhairpt.so && run base2 $L/libv_base/libhairpt.so
