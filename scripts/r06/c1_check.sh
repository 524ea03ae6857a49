#!/bin/bash
# C1 device tests + the kd leaf-size test, a headline bench (film fingerprint), the full-size C1 timing
set -o pipefail
mkdir -p gpurun_out/c1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c1.py tests/test_gpu_tree.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/c1/tree.log 2>&1
rc=$?
grep -E "stopPrims|oracle|passed|failed|Error|device vs" gpurun_out/c1/tree.log | cut -c1-700
[ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/c1/bench_splat.json 2> gpurun_out/c1/bench_splat.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/c1/bench_splat.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_ms_per_step'], repr(d['stats']['film_fingerprint']))"
timeout -k 10 300 python -u tools/c1_timing.py --width 1280 --height 720 --spp 64 --frames 3 > gpurun_out/c1/timing_full.json 2> gpurun_out/c1/timing_full.err || exit 1
cat gpurun_out/c1/timing_full.json
