# one-GPU strong-scaling rehearsal of C4 and C5 (the configs BASELINE assigns to 8 GPUs)
set -o pipefail
mkdir -p gpurun_out/reh
for c in curly_marschner furball_1m; do
  echo "== $c"
  timeout -k 10 600 python -u tools/shard_timing.py --config $c --reps 2 --ns 2,4,8 > gpurun_out/reh/$c.log 2>&1 || exit 1
  grep "ranks" gpurun_out/reh/$c.log | cut -c1-200
done
