# final check of the shipped build, as the driver runs it: pytest -m gpu, smoke, bench.py defaults
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final/gputests.log 2>&1 || { tail -40 gpurun_out/final/gputests.log; exit 1; }
tail -1 gpurun_out/final/gputests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log | cut -c1-200
timeout -k 10 600 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['stats']['film_fingerprint'])"
