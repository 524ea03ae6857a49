#!/bin/bash
# A/B kd-tree build parameters (hair shape kd* properties) on the bench workload.
# Usage: scripts/archive/kd_variants.sh "k=v,k=v" "k=v" ...
set -o pipefail
mkdir -p gpurun_out
for kd in "" "$@"; do
  timeout -k 10 200 python bench.py --cpu-baseline off --steps 2 --warmup 1 --kd "$kd" > gpurun_out/kd.log 2>&1 || { echo "FAIL $kd"; tail -5 gpurun_out/kd.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/kd.log').read().strip().splitlines()[-1])
print('%-45s %8.2f Mpaths/s trace %7.1f ms/step nodes/ray %.1f prims/ray %.1f exact/ray %.2f kd_nodes %d' % ('$kd' or 'default', d['value'], d['roofline']['rank0_trace_ms_per_step'], d['stats']['nodes_per_ray'], d['stats']['prims_per_ray'], d['stats']['exact_tests_per_ray'], d['config']['kd_nodes']))"
done
