# shadow-ray outcomes handed to post through P.sres (k_trace no longer adds NEE to li of a path that is posted): parity, bit-identity, bench
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_bounce_ahead.py > gpurun_out/r04/handoff_pytest.log 2>&1 || { tail -40 gpurun_out/r04/handoff_pytest.log; exit 1; }
tail -1 gpurun_out/r04/handoff_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_handoff.json 2> gpurun_out/r04/bench_handoff.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_handoff.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
