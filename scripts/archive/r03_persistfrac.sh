# persistent grids at 1/k of the resident slots (HPT_PERSIST_FRAC): N=8 shard and N=1
set -o pipefail
mkdir -p gpurun_out/pf
for K in 1 2; do
  echo "== frac $K"
  HPT_PERSIST_FRAC=$K timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/pf/pf$K.log 2>&1 || exit 1
  grep "^N=8" gpurun_out/pf/pf$K.log | cut -c1-260; grep '^{' gpurun_out/pf/pf$K.log | cut -c1-60
done
