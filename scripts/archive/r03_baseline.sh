# Round-3 baseline on the GPU box: smoke, headline bench, one-GPU strong-scaling rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err || exit 1
timeout -k 10 400 python -u tools/shard_timing.py --reps 3 > gpurun_out/r03_shards.log 2>&1 || exit 1
