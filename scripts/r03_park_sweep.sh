set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/park_sweep.log
for pr in 0 4 8 16 32; do
for pm in 524288 131072; do
echo "== rounds $pr parkmin $pm" >> gpurun_out/park_sweep.log
HPT_PARK_ROUNDS=$pr HPT_PARK_MIN=$pm timeout -k 10 120 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/ps.log 2>&1 || exit 1
grep -E "N=8 ranks|N1" gpurun_out/ps.log | sed 's/{"config.*N1_ms": \([0-9.]*\).*/N1 \1/' >> gpurun_out/park_sweep.log
done; done
