#!/bin/bash
# k_paths iteration: the bit-identity tests, then the headline bench with the phase report (k_paths on)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r06; mkdir -p $O
[ -n "$SKIPTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_paths.py -x -q --timeout 150 --timeout-method thread > $O/paths_test.log 2>&1
rc=$?; [ -n "$SKIPTEST" ] || { tail -3 $O/paths_test.log; [ $rc -eq 0 ] || exit $rc; }
HPT_PATHS=1 HPT_PATHS_REPORT=1 timeout -k 10 240 python -u bench.py --steps 3 --warmup 2 --cpu-baseline off > $O/it.json 2> $O/it.err || exit $?
python3 -c "import json; d=json.loads(open('$O/it.json').read().strip().splitlines()[-1]); print('paths', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
grep "\[paths\]" $O/it.err | tail -2
