# queue-ordered 4-byte hit records: the full GPU tier on the main build, the split variant's
# bit-exactness subset, then A/B bench and N=8 shard timing (main vs split)
set -o pipefail
mkdir -p gpurun_out/rec
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rec/gputests.log 2>&1 || { tail -40 gpurun_out/rec/gputests.log; exit 1; }
tail -2 gpurun_out/rec/gputests.log
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_split/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "trace_bit_exact or render_matches_oracle or tail_kernel or packet or full_size_headline" > gpurun_out/rec/split_pytest.log 2>&1 || { tail -40 gpurun_out/rec/split_pytest.log; exit 1; }
tail -2 gpurun_out/rec/split_pytest.log
bash scripts/archive/r03_variants.sh main split main split || exit 1
for V in main split; do
  if [ $V = main ]; then L2=""; else L2=$L; fi
  HAIRPT_LIB=$L2 timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/rec/shards_$V.log 2>&1 || exit 1
  echo "== $V"; grep "^N=8 rank 0\|^N=8 ranks" gpurun_out/rec/shards_$V.log | cut -c1-250
done
