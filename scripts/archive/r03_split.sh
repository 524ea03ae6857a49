# drain splitting (variants split*): bit-exactness through the variant, then A/B bench and N=8 shard timing
set -o pipefail
mkdir -p gpurun_out/split
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_split/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "trace_bit_exact or render_matches_oracle or tail_kernel" > gpurun_out/split/pytest.log 2>&1 || { tail -40 gpurun_out/split/pytest.log; exit 1; }
tail -3 gpurun_out/split/pytest.log
bash scripts/archive/r03_variants.sh main split || exit 1
for V in main ${VARS:-split main split}; do
  if [ $V = main ]; then L2=""; else L2=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so; fi
  HAIRPT_LIB=$L2 timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/split/shards_$V.log 2>&1 || exit 1
  echo "== $V"; grep "^N=8 rank 0\|^N=8 ranks" gpurun_out/split/shards_$V.log | cut -c1-250
done
