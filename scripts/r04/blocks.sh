# launch-shape variants (make variant): k_post 256-thread blocks, k_shade 128-thread blocks, camera / primary 256-thread blocks
set -o pipefail
mkdir -p gpurun_out/r04
for v in post256 shade128 q256; do
  HAIRPT_LIB=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --cpu-baseline off > gpurun_out/r04/blocks_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/blocks_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['kernel_ms_per_step'], d['stats']['film_fingerprint'])"
done
