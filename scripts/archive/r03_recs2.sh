# queue-ordered records, final form: GPU tier + smoke, then the one-GPU strong-scaling rehearsal
set -o pipefail
mkdir -p gpurun_out/recs2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/recs2/gputests.log 2>&1 || { tail -40 gpurun_out/recs2/gputests.log; exit 1; }
tail -1 gpurun_out/recs2/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/recs2/smoke.log 2>&1 || { tail -20 gpurun_out/recs2/smoke.log; exit 1; }
timeout -k 10 400 python -u tools/shard_timing.py --reps 2 > gpurun_out/recs2/shards.log 2>&1 || exit 1
grep "^N=\|^{" gpurun_out/recs2/shards.log | cut -c1-300
