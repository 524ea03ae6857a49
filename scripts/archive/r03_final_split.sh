# drain splitting on by default + queue-ordered hit records: GPU tier + smoke, A/B against the
# build without splitting, the one-GPU strong-scaling rehearsal, then the headline profile refresh
set -o pipefail
mkdir -p gpurun_out/fs
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fs/gputests.log 2>&1 || { tail -40 gpurun_out/fs/gputests.log; exit 1; }
tail -1 gpurun_out/fs/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fs/smoke.log 2>&1 || { tail -20 gpurun_out/fs/smoke.log; exit 1; }
tail -1 gpurun_out/fs/smoke.log
bash scripts/archive/r03_variants.sh main nosplit main nosplit || exit 1
timeout -k 10 400 python -u tools/shard_timing.py --reps 2 > gpurun_out/fs/shards.log 2>&1 || exit 1
grep "^N=\|^{" gpurun_out/fs/shards.log | cut -c1-300
bash scripts/archive/r03_configs.sh furball_marschner || exit 1
