# k_tail occupancy (HPT_TAIL_WAVES 2/4/5 variant builds): the tail for everything after the camera pass
set -o pipefail
mkdir -p gpurun_out/tailwaves
for V in main tail4 tail5; do
  if [ $V = main ]; then L=""; else L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so; fi
  for T in 1048576 2097152 4194304; do
    echo "== $V tail $T"
    HAIRPT_LIB=$L HPT_TAIL_PATHS=$T timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/tailwaves/${V}_$T.log 2>&1 || exit 1
    grep "^N=8 rank 0\|^N=8 ranks" gpurun_out/tailwaves/${V}_$T.log | cut -c1-250
  done
done
