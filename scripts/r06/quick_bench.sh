#!/bin/bash
# a headline bench at the current build: value, ms per frame, the per-kernel split and the film fingerprint
# (the exact-arithmetic fp64 sum of the frame: unchanged = bit-identical films); optional pytest -k filter
set -o pipefail
mkdir -p gpurun_out/qb
if [ -n "$1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$1" --timeout 300 --timeout-method thread > gpurun_out/qb/tests.log 2>&1 || { tail -30 gpurun_out/qb/tests.log; exit 1; }
  tail -1 gpurun_out/qb/tests.log
fi
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/qb/bench.json 2> gpurun_out/qb/bench.err || { tail -20 gpurun_out/qb/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/qb/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], repr(d['stats']['film_fingerprint']))"
