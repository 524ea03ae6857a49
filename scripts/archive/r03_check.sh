# correctness + timing check: headline bench (fingerprint), one-GPU rehearsal, GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/chk_bench.json 2> gpurun_out/chk.err || exit 1
timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 2,4,8 > gpurun_out/chk_shards.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk_pytest.log 2>&1 || exit 1
