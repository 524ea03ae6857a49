#!/bin/bash
# k_paths (persistent bounce kernel): bit-identity tests against the wavefront loop, then the
# headline bench with k_paths on (default) and off (HPT_PATHS=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
O=gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -x -v --timeout 150 --timeout-method thread > $O/paths_test.log 2>&1
rc=$?
tail -5 $O/paths_test.log
[ $rc -eq 0 ] || exit $rc
HPT_PATHS=1 timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/bench_paths.json 2> $O/bench_paths.err || exit $?
HPT_PATHS=0 timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/bench_wave.json 2> $O/bench_wave.err || exit $?
python - <<'PY'
import json
for f in ("bench_paths", "bench_wave"):
    d = json.loads(open("gpurun_out/r06/%s.json" % f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["kernel_ms_per_step"], d["stats"]["film_fingerprint"])
PY
