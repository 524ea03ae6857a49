# the driver's round-end commands: the whole GPU test suite, smoke(), the default bench line
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/final_pytest.log 2>&1 || { tail -40 gpurun_out/r04/final_pytest.log; exit 1; }
tail -2 gpurun_out/r04/final_pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/final_smoke.log 2>&1 || { tail -20 gpurun_out/r04/final_smoke.log; exit 1; }
tail -2 gpurun_out/r04/final_smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/r04/final_bench.json 2> gpurun_out/r04/final_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/final_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
