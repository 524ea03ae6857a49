# resumable cut: bit-identity tests, then the headline bench and the N=8 rehearsal (cut on / off)
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_bounce_ahead.py > gpurun_out/r05/cut_pytest.log 2>&1 || { tail -60 gpurun_out/r05/cut_pytest.log; exit 1; }
tail -3 gpurun_out/r05/cut_pytest.log
for C in 0 262144; do
  HPT_CUT_MIN=$C timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r05/cut_bench_$C.json 2> gpurun_out/r05/cut_bench_$C.err || exit 1
  tail -1 gpurun_out/r05/cut_bench_$C.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cut_min $C', d['value'], d['ms_per_step'], d['stats']['film_fingerprint'], d['stats'].get('cut_rays'))"
  HPT_CUT_MIN=$C timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance --stats-level 0 > gpurun_out/r05/cut_reh_$C.txt 2>&1 || exit 1
  echo "cut_min $C: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/cut_reh_$C.txt) $(grep 'N=8 ranks' gpurun_out/r05/cut_reh_$C.txt | grep -o 'max.*')"
done
