#!/bin/bash
# camera rays from the film position: parity tests, then bench A/B of four builds on one box
# (base: before this round's pre-test classes; head: classes; main: classes + camera change;
#  glob: main with one global pre-test radius)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_camera.py tests/test_gpu_bounce_ahead.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/cam_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error" $O/cam_tests.log | tail -5; [ $rc -eq 0 ] || exit $rc
L=$PWD/cs184-final-project-mitsuba0.5_amd
run() { # name lib
  HAIRPT_LIB=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/cab_$1.json 2> $O/cab_$1.err || return $?
  python3 - $1 <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/r06/cab_%s.json" % v).read().strip().splitlines()[-1])
k = d["roofline"].get("kernel_ms_per_step") or {}
print(v, d["value"], d["ms_per_step"], d["roofline"].get("rank0_trace_ms_per_step"), d["stats"]["exact_tests_per_ray"],
      d["stats"].get("film_fingerprint"), {x: k.get(x) for x in ("camera", "trace_packet", "primary", "trace")})
PY
}
run base $L/libv_base/libhairpt.so && run head $L/libv_head/libhairpt.so && run main $L/lib/libhairpt.so && run glob $L/libv_glob/libhairpt.so && run main2 $L/lib/libhairpt.so && run base2 $L/libv_base/libhairpt.so
