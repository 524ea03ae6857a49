#!/bin/bash
# Round-2 evidence run (on the GPU box through gpurun, from the repo root):
#   rocprofv3 kernel trace + FETCH/WRITE passes, the PMC groups of gpu_pmc.sh, and the
#   one-GPU strong-scaling rehearsal of every rank (tools/shard_timing.py --all-ranks).
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r02}
bash "$ROOT/scripts/gpu_profile.sh" "$TAG" --steps 3 --warmup 1
bash "$ROOT/scripts/gpu_pmc.sh" "$TAG" --steps 3 --warmup 1
cd "$ROOT"
timeout -k 10 300 python3 tools/shard_timing.py --all-ranks > gpurun_out/shards_$TAG.json 2> gpurun_out/shards_$TAG.err
echo "r02 profile done"
