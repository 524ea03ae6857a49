# launch cut with block-aggregated carry appends: tests, N=8 rehearsal and headline for cut off / on / on after a partial drain
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cut.py tests/test_gpu_bounce_ahead.py > gpurun_out/r04/cut2_pytest.log 2>&1 || { tail -40 gpurun_out/r04/cut2_pytest.log; exit 1; }
tail -2 gpurun_out/r04/cut2_pytest.log
for V in "0 0" "1 0" "1 100" "1 250"; do
  set -- $V
  HPT_CUT=$1 HPT_CUT_AFTER_US=$2 timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 > gpurun_out/r04/reh2_c$1_a$2.txt 2>&1 || exit 1
  echo "cut=$1 after=$2"; grep "N=8" gpurun_out/r04/reh2_c$1_a$2.txt
  HPT_CUT=$1 HPT_CUT_AFTER_US=$2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r04/bench2_c$1_a$2.json 2> gpurun_out/r04/bench2_c$1_a$2.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/bench2_c$1_a$2.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'], d['first_render_ms'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'], d['stats']['cut_rays_per_frame'])"
done
