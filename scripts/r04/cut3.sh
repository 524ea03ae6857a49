# lane-level launch cut (closest rays to the next launch, the wave's idle lanes help its shadow rays):
# bit-identity, then the N=8 rehearsal cut off / on for the shipped build and two scheduler variants
set -o pipefail
mkdir -p gpurun_out/r04
for V in ilp; do
  L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so
  HAIRPT_LIB=$L timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r04/cut3_pytest_$V.log 2>&1 || { tail -30 gpurun_out/r04/cut3_pytest_$V.log; exit 1; }
  tail -1 gpurun_out/r04/cut3_pytest_$V.log
done
for V in lib ilp; do
  if [ $V = lib ]; then L=$(pwd)/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so; fi
  for C in 0 1; do
    HPT_CUT=$C HAIRPT_LIB=$L timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/reh3_${V}_c$C.txt 2>&1 || exit 1
    echo "$V cut=$C N1 $(python3 -c "import json,re; t=open('gpurun_out/r04/reh3_${V}_c$C.txt').read(); print(re.findall(r'\"N1_ms\": ([0-9.]+)', t))")"; grep "N=8" gpurun_out/r04/reh3_${V}_c$C.txt
  done
done
