#!/bin/bash
# k_paths phase statistics at the headline frame for backlog-control variants (HPT_PATHS_REPORT)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HPT_PATHS_REPORT=1 HPT_PATHS=1
O=gpurun_out/r06; mkdir -p $O
run() { # name env...
  local n=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 2 --warmup 2 --cpu-baseline off > $O/probe_$n.json 2> $O/probe_$n.err || return $?
  python3 -c "import json,sys; d=json.loads(open('$O/probe_$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'])"
  grep "\[paths\]" $O/probe_$n.err | tail -1
}
run base || exit $?
run low8 HPT_PATHS_LOW=8 HPT_PATHS_HIGH=16 || exit $?
run sh32 HPT_PATHS_SHADERS=32 || exit $?
run sh4 HPT_PATHS_SHADERS=4 HPT_PATHS_LOW=1 HPT_PATHS_HIGH=2 || exit $?
