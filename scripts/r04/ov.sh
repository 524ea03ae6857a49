# overlapped bounces (k_post_early beside k_trace): bit-identity tests, bench with/without, N=8 rehearsal, N=8 kernel trace
set -o pipefail
mkdir -p gpurun_out/r04/ovtl
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_overlap.py > gpurun_out/r04/ov_pytest.log 2>&1 || { tail -40 gpurun_out/r04/ov_pytest.log; exit 1; }
tail -1 gpurun_out/r04/ov_pytest.log
for o in 0 1; do
  HPT_OVERLAP=$o timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_ov$o.json 2> gpurun_out/r04/bench_ov$o.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_ov$o.json').read().strip().splitlines()[-1]); print('overlap $o bench', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
done
HPT_OVERLAP=1 timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/reh_ov.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/reh_ov.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HPT_OVERLAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/ovtl -o tl -- python3 tools/shard_timing.py --reps 3 --ns 8 --balance > gpurun_out/r04/ovtl.log 2>&1 || { tail -20 gpurun_out/r04/ovtl.log; exit 1; }
find gpurun_out/r04/ovtl -name "*kernel_trace.csv" | head -3
