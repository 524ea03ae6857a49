set -o pipefail
mkdir -p gpurun_out
HPT_BOUNCE_REPORT=1 timeout -k 10 300 python -u tools/shard_timing.py --reps 1 > gpurun_out/bounces.log 2>&1 || exit 1
HPT_PARK_MIN=0 HPT_BOUNCE_REPORT=1 timeout -k 10 300 python -u tools/shard_timing.py --reps 1 > gpurun_out/bounces_nopark.log 2>&1 || exit 1
