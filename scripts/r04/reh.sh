# one-GPU scaling rehearsal at the current build (balanced deal), N = 2, 4, 8
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance > gpurun_out/r04/reh_final.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/reh_final.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
