# one-GPU N=2,4,8 strong-scaling rehearsals (every rank, balanced deal) of the given configs
set -o pipefail
mkdir -p gpurun_out/r06cfg
for c in "$@"; do
  echo "== $c"
  timeout -k 10 500 python -u tools/shard_timing.py --config $c --all-ranks --reps 2 --ns 2,4,8 --balance > gpurun_out/r06cfg/reh_$c.txt 2>&1 || exit 1
  grep "ranks" gpurun_out/r06cfg/reh_$c.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
done
