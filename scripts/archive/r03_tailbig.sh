# k_tail taking over earlier: one-GPU rehearsal at N=8 for large HPT_TAIL_PATHS thresholds
set -o pipefail
mkdir -p gpurun_out/tailbig
for T in 131072 1048576 4194304 16777216; do
  echo "== tail $T"
  HPT_TAIL_PATHS=$T timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/tailbig/shards_$T.log 2>&1 || exit 1
  grep "^N=8" gpurun_out/tailbig/shards_$T.log | cut -c1-300
done
