# k_trace launch timelines, rank 0 of 8: the shipped traversal vs drain splitting
set -o pipefail
mkdir -p gpurun_out/splitprof
for V in traceprof splitprof; do
  L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so
  HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/splitprof/$V.jsonl 2> gpurun_out/splitprof/$V.err || exit 1
  echo "== $V"; cat gpurun_out/splitprof/$V.jsonl
done
