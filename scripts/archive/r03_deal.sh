set -o pipefail
mkdir -p gpurun_out/deal
for k in 1 2 4; do
  HPT_DEAL_CHUNK=$k timeout -k 10 300 python -u tools/shard_timing.py --all-ranks --ns 8 > gpurun_out/deal/shards_$k.log 2>&1 || { tail -20 gpurun_out/deal/shards_$k.log; exit 1; }
  echo "chunk=$k"; grep -E "ranks|rank 0 kernels" gpurun_out/deal/shards_$k.log | cut -c1-400
done
