# dump launches 1 and 3 of the N=8 shard's ray costs for offline claim-order modelling
set -o pipefail
mkdir -p gpurun_out/r04
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_raylog/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u tools/ray_order_probe.py --shards 8 --no-sim --dump gpurun_out/r04/raydump_n8.npz > gpurun_out/r04/raydump.jsonl 2> gpurun_out/r04/raydump.err || { tail -20 gpurun_out/r04/raydump.err; exit 1; }
ls -la gpurun_out/r04/raydump_n8.npz
