# claim-order buckets (longest rays claimed first) at the N=8 shard, balanced deal
set -o pipefail
mkdir -p gpurun_out/r04
for B in 0 1; do
  HPT_CLAIM_BUCKETS=$B timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/bk_$B.txt 2>&1 || exit 1
  echo "buckets=$B $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r04/bk_$B.txt) $(grep 'N=8 ranks' gpurun_out/r04/bk_$B.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r04/bk_$B.txt | cut -c1-220
done
