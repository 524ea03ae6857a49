# post fused with the next bounce's shading (k_postshade): bounce-ahead / fused bit-identity, parity, bench fused / unfused, N=8 rehearsal
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_bounce_ahead.py tests/test_gpu_parity.py > gpurun_out/r04/fuse_pytest.log 2>&1 || { tail -40 gpurun_out/r04/fuse_pytest.log; exit 1; }
tail -1 gpurun_out/r04/fuse_pytest.log
for f in 0 1; do
  HPT_FUSE=$f timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_fuse$f.json 2> gpurun_out/r04/bench_fuse$f.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_fuse$f.json').read().strip().splitlines()[-1]); print('fuse $f bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
done
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance > gpurun_out/r04/reh_fuse.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/reh_fuse.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
