# launch cut: bit-identity tests, headline bench with the cut on / off (and camera rays without packets),
# N=8 one-GPU rehearsal on / off, rocprofv3 kernel summary of the cut build
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_bounce_ahead.py tests/test_gpu_balance.py tests/test_gpu_distributed.py > gpurun_out/r04/cut_pytest.log 2>&1 || { tail -40 gpurun_out/r04/cut_pytest.log; exit 1; }
tail -3 gpurun_out/r04/cut_pytest.log
for C in 1 0; do
  HPT_CUT=$C timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_cut$C.json 2> gpurun_out/r04/bench_cut$C.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_cut$C.json').read().strip().splitlines()[-1]); print('cut=$C', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'], d['stats']['cut_rays_per_frame'])"
done
for C in 1 0; do
  HPT_CUT=$C timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/rehearsal_cut$C.txt 2>&1 || exit 1
  grep "N=8" gpurun_out/r04/rehearsal_cut$C.txt
done
HPT_CUT=1 timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r04/rehearsal_cut1_bal.txt 2>&1 || exit 1
grep "N=8" gpurun_out/r04/rehearsal_cut1_bal.txt
HPT_CUT=1 HPT_PACKETS=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench_nopk.json 2> gpurun_out/r04/bench_nopk.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench_nopk.json').read().strip().splitlines()[-1]); print('no packets', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
HPT_CUT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/prof_cut -o run -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/r04/prof_cut.log 2>&1 || exit 1
find gpurun_out/r04/prof_cut -name "*stats*" | head
