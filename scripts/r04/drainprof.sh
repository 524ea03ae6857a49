# k_trace drain anatomy at the current build: per-launch wave exits after the dry point,
# drain-loop rounds and lane use (traceprof variant), rank 0 of 8 and of 1; then the
# shipped library's one-GPU scaling rehearsal (all ranks)
set -o pipefail
mkdir -p gpurun_out/r04
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_traceprof/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/r04/drain_n8.jsonl 2> gpurun_out/r04/drain_n8.err || exit 1
HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 1 > gpurun_out/r04/drain_n1.jsonl 2> gpurun_out/r04/drain_n1.err || exit 1
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 > gpurun_out/r04/rehearsal_base.txt 2>&1 || exit 1
cat gpurun_out/r04/rehearsal_base.txt
