# A/B of ray parking: headline bench film fingerprint and time with parking off / on, then the one-GPU rehearsal
set -o pipefail
mkdir -p gpurun_out
HPT_PARK_MIN=0 timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/park_off.json 2> gpurun_out/park.err || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/park_on.json 2>> gpurun_out/park.err || exit 1
timeout -k 10 400 python -u tools/shard_timing.py --reps 3 > gpurun_out/park_shards.log 2>&1 || exit 1
