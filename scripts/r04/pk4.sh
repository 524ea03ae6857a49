# camera packets over the two-level records: packet / trace parity tests, headline bench, N=8 rehearsal
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r04/pk4_pytest.log 2>&1 || { tail -40 gpurun_out/r04/pk4_pytest.log; exit 1; }
tail -1 gpurun_out/r04/pk4_pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_pk4.json 2> gpurun_out/r04/bench_pk4.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_pk4.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'], d['roofline_packet'])"
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/reh_pk4.txt 2>&1 || exit 1
grep "N=8\|N1_ms" gpurun_out/r04/reh_pk4.txt | cut -c1-300
