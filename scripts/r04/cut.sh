# launch cut: bit-identity tests, headline bench with the cut on / off, N=8 one-GPU rehearsal on / off
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_bounce_ahead.py tests/test_gpu_balance.py > gpurun_out/r04/cut_pytest.log 2>&1 || { tail -40 gpurun_out/r04/cut_pytest.log; exit 1; }
tail -3 gpurun_out/r04/cut_pytest.log
for C in 1 0; do
  HPT_CUT=$C timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_cut$C.json 2> gpurun_out/r04/bench_cut$C.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_cut$C.json').read().strip().splitlines()[-1]); print('cut=$C', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'], d['stats']['cut_rays_per_frame'])"
done
for C in 1 0; do
  HPT_CUT=$C timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/rehearsal_cut$C.txt 2>&1 || exit 1
  grep "N=8" gpurun_out/r04/rehearsal_cut$C.txt
done
