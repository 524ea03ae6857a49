# one-GPU strong-scaling rehearsal: Hilbert-cyclic block deal (bench.py) vs an spp split of every pixel
set -o pipefail
mkdir -p gpurun_out/split
for m in blocks spp; do
  timeout -k 10 300 python -u tools/shard_timing.py --all-ranks --split $m > gpurun_out/split/shards_$m.log 2>&1 || { tail -20 gpurun_out/split/shards_$m.log; exit 1; }
  echo "split=$m"; grep -E "ranks|rank 0 kernels" gpurun_out/split/shards_$m.log | cut -c1-400
done
