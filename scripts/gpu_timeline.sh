#!/bin/bash
# Kernel timeline of one N=8 shard frame (rocprofv3 kernel trace), for the scaling analysis.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/timeline_${TAG:-r02}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/db" -o tl -- python3 "$ROOT/tools/launch_timeline.py" --n ${N:-8} > "$OUT/run.log" 2>&1
echo "timeline done"
