# k_tail threshold at the N=8 shard (balanced deal): 2^14 / 2^15 / 2^16 / 2^17 (shipped) live paths
set -o pipefail
mkdir -p gpurun_out/r04
for T in 16384 32768 65536 131072; do
  HPT_TAIL_PATHS=$T timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/tt_$T.txt 2>&1 || exit 1
  echo "tail=$T $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r04/tt_$T.txt) $(grep 'N=8 ranks' gpurun_out/r04/tt_$T.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r04/tt_$T.txt | cut -c1-220
done
