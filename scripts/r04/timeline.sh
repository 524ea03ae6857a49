# kernel timeline of the N=8 shard (balanced deal) under rocprofv3 --kernel-trace: per-launch durations and gaps
set -o pipefail
mkdir -p gpurun_out/r04/tl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/tl -o tl -- python3 tools/shard_timing.py --reps 3 --ns 8 --balance > gpurun_out/r04/tl.log 2>&1 || { tail -20 gpurun_out/r04/tl.log; exit 1; }
find gpurun_out/r04/tl -name "*kernel_trace.csv" | head -3
