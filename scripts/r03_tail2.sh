set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tail2.log
HPT_PARK_MIN=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/t2_off.json 2> gpurun_out/t2.err || exit 1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/t2_on.json 2>> gpurun_out/t2.err || exit 1
for tp in 131072 262144 524288; do
for pr in 8 1000000; do
echo "== tail $tp parkrounds $pr" >> gpurun_out/tail2.log
HPT_TAIL_PATHS=$tp HPT_PARK_ROUNDS=$pr timeout -k 10 120 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/ps.log 2>&1 || exit 1
grep -E "N=8 ranks|N1" gpurun_out/ps.log | sed 's/{"config.*N1_ms": \([0-9.]*\).*/N1 \1/' >> gpurun_out/tail2.log
done; done
HPT_BOUNCE_REPORT=1 timeout -k 10 120 python -u tools/shard_timing.py --reps 1 --ns 8 > gpurun_out/t2_bounces.log 2>&1 || exit 1
