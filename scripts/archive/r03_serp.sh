# one-GPU strong-scaling rehearsal: Hilbert-cyclic deal vs boustrophedon (odd rounds dealt in reverse)
set -o pipefail
mkdir -p gpurun_out/serp
for m in 0 1; do
  HPT_DEAL_SERP=$m timeout -k 10 300 python -u tools/shard_timing.py --all-ranks > gpurun_out/serp/shards_$m.log 2>&1 || { tail -20 gpurun_out/serp/shards_$m.log; exit 1; }
  echo "serp=$m"; grep -E "ranks" gpurun_out/serp/shards_$m.log | cut -c1-400
done
