# ray-cost predictors and a claim-order model of k_trace's drain (tools/ray_order_probe.py)
set -o pipefail
mkdir -p gpurun_out/r04
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_raylog/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 900 python -u tools/ray_order_probe.py --shards 8 > gpurun_out/r04/raylog_n8.jsonl 2> gpurun_out/r04/raylog_n8.err || { tail -20 gpurun_out/r04/raylog_n8.err; exit 1; }
cat gpurun_out/r04/raylog_n8.jsonl | cut -c1-600
