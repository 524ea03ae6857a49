set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tailk.log
for pr in 16 32 64 128; do
echo "== parkrounds $pr" >> gpurun_out/tailk.log
HPT_PARK_ROUNDS=$pr timeout -k 10 120 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/ps.log 2>&1 || exit 1
grep -E "N=8 ranks|N=8 rank 0|N1" gpurun_out/ps.log | sed 's/{"config.*N1_ms": \([0-9.]*\).*/N1 \1/' >> gpurun_out/tailk.log
done
