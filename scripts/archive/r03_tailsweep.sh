# k_tail threshold sweep (live paths below which the frame's remaining bounces run in k_tail)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/tailsweep.log
for tp in 65536 131072 262144 524288 1048576; do
echo "== tail $tp" >> gpurun_out/tailsweep.log
HPT_TAIL_PATHS=$tp timeout -k 10 120 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/ps.log 2>&1 || exit 1
grep -E "N=8 ranks|N=8 rank 0|N1" gpurun_out/ps.log | sed 's/{"config.*N1_ms": \([0-9.]*\).*/N1 \1/' >> gpurun_out/tailsweep.log
done
