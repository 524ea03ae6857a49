# striped block-cost counters: balance test, headline bench (packets on / off), N=8 rehearsal (Hilbert / balanced deal)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_balance.py tests/test_gpu_bounce_ahead.py > gpurun_out/r04/stripes_pytest.log 2>&1 || { tail -40 gpurun_out/r04/stripes_pytest.log; exit 1; }
tail -3 gpurun_out/r04/stripes_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_s.json 2> gpurun_out/r04/bench_s.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_s.json').read().strip().splitlines()[-1]); print('stripes', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
HPT_PACKETS=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_nopk.json 2> gpurun_out/r04/bench_nopk.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_nopk.json').read().strip().splitlines()[-1]); print('no packets', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/rehearsal_s.txt 2>&1 || exit 1
grep "N=8" gpurun_out/r04/rehearsal_s.txt
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/rehearsal_sbal.txt 2>&1 || exit 1
grep "N=8" gpurun_out/r04/rehearsal_sbal.txt
