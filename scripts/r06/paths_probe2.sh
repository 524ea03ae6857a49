#!/bin/bash
# k_paths: global words read once per chunk (default build, MachineLICM off) vs the MachineLICM-on variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HPT_PATHS_REPORT=1 HPT_PATHS=1
O=gpurun_out/r06; mkdir -p $O
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 2 --warmup 2 --cpu-baseline off > $O/probe_$n.json 2> $O/probe_$n.err || return $?
  python3 -c "import json,sys; d=json.loads(open('$O/probe_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['stats']['film_fingerprint'])"
  grep "\[paths\]" $O/probe_$n.err | tail -1
}
run once || exit $?
run licm HAIRPT_LIB=cs184-final-project-mitsuba0.5_amd/libv_licm/libhairpt.so || exit $?
