#!/bin/bash
# A/B the kernel variant builds (libv_*/libhairpt.so) on the bench workload.
set -o pipefail
mkdir -p gpurun_out
for v in lib "$@"; do
  if [ "$v" = lib ]; then lib=cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else lib=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$PWD/$lib timeout -k 10 200 python bench.py --cpu-baseline off --steps 2 --warmup 1 $BENCH_ARGS > gpurun_out/var.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/var.log; exit 1; }
  python -c "
import json
d=json.loads(open('gpurun_out/var.log').read().strip().splitlines()[-1])
print('%-10s %8.2f Mpaths/s trace %7.1f ms/step %.1f GB/s nodes/ray %.1f prims/ray %.1f film %.9e' % ('$v', d['value'], d['roofline']['rank0_trace_ms_per_step'], d['roofline']['achieved'], d['stats']['nodes_per_ray'], d['stats']['prims_per_ray'], d['stats'].get('film_fingerprint', 0)))"
done
