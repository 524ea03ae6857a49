# drain parameters at the N=8 shard (balanced deal): HPT_SPLIT_MIN 2 / 4 / 8 (shipped), HPT_REFILL 8 / 16 (shipped) / 32,
# and k_tail without idle-lane splitting
set -o pipefail
mkdir -p gpurun_out/r04
for V in lib split2 split4 refill8 refill32 tailnosplit; do
  if [ $V = lib ]; then L=$(pwd)/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so; fi
  HAIRPT_LIB=$L timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/dv_$V.txt 2>&1 || exit 1
  echo "$V $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r04/dv_$V.txt) $(grep 'N=8 ranks' gpurun_out/r04/dv_$V.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r04/dv_$V.txt | cut -c1-220
done
