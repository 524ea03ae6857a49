# the whole GPU tier at the current build, then smoke() and a short headline bench
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/gputests.log 2>&1 || { tail -40 gpurun_out/r06/gputests.log; exit 1; }
tail -2 gpurun_out/r06/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || { tail -20 gpurun_out/r06/smoke.log; exit 1; }
tail -2 gpurun_out/r06/smoke.log
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/r06/bench_check.json 2> gpurun_out/r06/bench_check.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r06/bench_check.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'])"
