# claim-order buckets + work-balanced deal: bit-identity tests (claim order, bounce-ahead,
# multi-device, C ABI, balance), then the headline bench with buckets off / on, and the N=8
# one-GPU rehearsal: buckets off / on, and the work-balanced deal
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_claim_order.py tests/test_gpu_bounce_ahead.py tests/test_multi_device.py tests/test_c_abi.py tests/test_gpu_balance.py tests/test_gpu_parity.py > gpurun_out/r04/buckets_pytest.log 2>&1 || { tail -40 gpurun_out/r04/buckets_pytest.log; exit 1; }
tail -3 gpurun_out/r04/buckets_pytest.log
for B in 0 1; do
  HPT_CLAIM_BUCKETS=$B timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_b$B.json 2> gpurun_out/r04/bench_b$B.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_b$B.json').read().strip().splitlines()[-1]); print('B=$B', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
done
HPT_PACKETS=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_nopk.json 2> gpurun_out/r04/bench_nopk.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_nopk.json').read().strip().splitlines()[-1]); print('no packets', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
for B in 0 1; do
  HPT_CLAIM_BUCKETS=$B timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/rehearsal_b$B.txt 2>&1 || exit 1
  grep "N=8 ranks" gpurun_out/r04/rehearsal_b$B.txt
done
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/rehearsal_bal.txt 2>&1 || exit 1
grep "N=8 ranks" gpurun_out/r04/rehearsal_bal.txt
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_tailnosplit/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/rehearsal_tailnosplit.txt 2>&1 || exit 1
grep "N=8 ranks" gpurun_out/r04/rehearsal_tailnosplit.txt
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --stats-level 0 > gpurun_out/r04/rehearsal_nostats.txt 2>&1 || exit 1
grep "N=8 ranks" gpurun_out/r04/rehearsal_nostats.txt
