# work-balanced deal (path-bounces per block) vs Hilbert-cyclic at N=2,4,8 on the headline config
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance bounces > gpurun_out/r04/bal_bounces.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/bal_bounces.txt | cut -c1-400
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance > gpurun_out/r04/bal_on.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/bal_on.txt | cut -c1-400
