#!/bin/bash
# Round profiling recipe (run on the GPU box through gpurun from the repo root):
#   1. rocprofv3 kernel trace + stats of the headline bench
#   2. separate PMC passes for HBM bytes (FETCH_SIZE, WRITE_SIZE cannot share a pass)
# Usage: scripts/gpu_profile.sh <tag> [bench args...]
set -eo pipefail
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench -- \
    python3 "$ROOT/bench.py" --cpu-baseline off "$@" > "$OUT/bench_trace.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o bench -- \
    python3 "$ROOT/bench.py" --cpu-baseline off "$@" > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o bench -- \
    python3 "$ROOT/bench.py" --cpu-baseline off "$@" > "$OUT/bench_write.log" 2>&1
echo "profile $TAG done"
