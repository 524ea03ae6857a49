# does per-kernel HIP event timing in the timed frames cost the N=8 shard? stats level 1 vs 0
set -o pipefail
mkdir -p gpurun_out/r05
for L in 1 0; do
  timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance --stats-level $L > gpurun_out/r05/evt_l$L.txt 2>&1 || exit 1
  echo "level $L: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/evt_l$L.txt) $(grep 'N=8 ranks' gpurun_out/r05/evt_l$L.txt | grep -o 'max.*')"
done
