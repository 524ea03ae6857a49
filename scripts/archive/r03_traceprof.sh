# k_trace launch timelines (variant build -DHPT_TRACE_PROFILE): N=1 and rank 0 of 8
set -o pipefail
mkdir -p gpurun_out/traceprof
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_traceprof/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/traceprof/n8.jsonl 2> gpurun_out/traceprof/n8.err || exit 1
HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 1 > gpurun_out/traceprof/n1.jsonl 2> gpurun_out/traceprof/n1.err || exit 1
cat gpurun_out/traceprof/n8.jsonl gpurun_out/traceprof/n1.jsonl
