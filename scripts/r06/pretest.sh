#!/bin/bash
# per-record pre-test classes: trace bit-exactness + the fold scene test, then the headline bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py::test_folded_strands_match_oracle_and_keep_the_pretest \
  tests/test_gpu_parity.py -x -v -s --timeout 300 --timeout-method thread > $O/pretest_tests.log 2>&1
rc=$?; grep -E "passed|failed|folded|fold-free|Error" $O/pretest_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/pretest_bench.json 2> $O/pretest_bench.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06/pretest_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"].get("rank0_trace_ms_per_step"), d["stats"]["exact_tests_per_ray"], d["stats"].get("film_fingerprint"))
PY
# cost probes of the node-record redesign: +16 B per node fetch, +1 dependent fetch per leaf
for v in pad lrt; do
  HAIRPT_LIB=$PWD/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --cpu-baseline off > $O/probe_$v.json 2> $O/probe_$v.err || exit $?
  python3 - $v <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open("gpurun_out/r06/probe_%s.json" % v).read().strip().splitlines()[-1])
print(v, d["value"], d["ms_per_step"], d["roofline"].get("rank0_trace_ms_per_step"), d["stats"]["exact_tests_per_ray"], d["stats"].get("film_fingerprint"))
PY
done
