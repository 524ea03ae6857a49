# one-GPU N=2,4,8 rehearsal of the headline at the current build (every rank, balanced deal)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance > gpurun_out/r06/reh_${1:-final}.txt 2>&1 || exit 1
grep "ranks\|N1_ms" gpurun_out/r06/reh_${1:-final}.txt | grep -o "N=[0-9] ranks.*\|\"N1_ms.*" | sed 's/{.*}//' | cut -c1-200
