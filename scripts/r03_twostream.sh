set -o pipefail
mkdir -p gpurun_out
HPT_PARK_MIN=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/ts_off.json 2> gpurun_out/ts.err || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/ts_on.json 2>> gpurun_out/ts.err || exit 1
HPT_BOUNCE_REPORT=1 timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 2,4,8 > gpurun_out/ts_shards.log 2>&1 || exit 1
