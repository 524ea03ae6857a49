# bounce queues keyed by direction octant within a k_shade block: parity, tail bit-identity, bench, N=8 rehearsal
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bounce_ahead.py tests/test_camera.py -m gpu > gpurun_out/r04/octq_pytest.log 2>&1 || { tail -40 gpurun_out/r04/octq_pytest.log; exit 1; }
tail -1 gpurun_out/r04/octq_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_octq.json 2> gpurun_out/r04/bench_octq.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_octq.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/reh_octq.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/reh_octq.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
