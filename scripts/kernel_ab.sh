# A/B per-kernel times of variant builds: bash scripts/kernel_ab.sh v1 v2 ...
set -o pipefail
for v in lib "$@"; do
  if [ $v = lib ]; then L=cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$PWD/$L timeout -k 10 300 python bench.py --cpu-baseline off --steps 2 --warmup 1 > gpurun_out/kab.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/kab.log').read().strip().splitlines()[-1]); print('%-8s %8.2f' % ('$v', d['value']), d['kernel_ms_per_step'], d['stats']['bounces_per_path'])"
done
