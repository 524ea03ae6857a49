set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/tl_shards.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/tl8/db -o tl -- python3 $GRAFT_REPO_ROOT/tools/launch_timeline.py --n 8 > $GRAFT_REPO_ROOT/gpurun_out/tl8.log 2>&1 || exit 1
