#!/bin/bash
# k_paths timing variants (phase report): plain (non-coherent) hand-off accesses, 2 entries, backlog knobs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HPT_PATHS=1 HPT_PATHS_REPORT=1
O=gpurun_out/r06; mkdir -p $O
L=cs184-final-project-mitsuba0.5_amd
run() { local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 2 --warmup 2 --cpu-baseline off > $O/v_$n.json 2> $O/v_$n.err || { echo "$n failed"; tail -3 $O/v_$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/v_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['stats']['film_fingerprint'])"
  grep "\[paths\]" $O/v_$n.err | tail -2; }
run plain HAIRPT_LIB=$L/libv_plain/libhairpt.so
run e2 HAIRPT_LIB=$L/libv_e2/libhairpt.so
run hi HPT_PATHS_LOW=8 HPT_PATHS_HIGH=16 HPT_PATHS_SHADERS=32
run sh8 HPT_PATHS_SHADERS=8
