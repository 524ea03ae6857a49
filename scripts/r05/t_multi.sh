# multi-device boundary tests + headline bench after the bucket removal
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multi_device.py tests/test_c_abi.py tests/test_gpu_balance.py tests/test_gpu_bounce_ahead.py > gpurun_out/r05/t_multi.log 2>&1 || { tail -40 gpurun_out/r05/t_multi.log; exit 1; }
tail -3 gpurun_out/r05/t_multi.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r05/bench_nobuckets.json 2> gpurun_out/r05/bench_nobuckets.err || exit 1
tail -1 gpurun_out/r05/bench_nobuckets.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('fingerprint', d.get('film_fingerprint')))"
