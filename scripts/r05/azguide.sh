# guided azimuthal cdf search: BSDF / render parity on the guided build, then the headline bench on the
# guided build and on the bisection build (HPT_AZ_BISECT): same film fingerprint, per-kernel times
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "bsdf or marschner or furball" > gpurun_out/r05/azguide_tests.log 2>&1 || { tail -30 gpurun_out/r05/azguide_tests.log; exit 1; }
tail -1 gpurun_out/r05/azguide_tests.log
for v in lib bis; do
  if [ $v = lib ]; then L=$PWD/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=$PWD/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$L timeout -k 10 300 python bench.py --cpu-baseline off --steps 3 --warmup 1 > gpurun_out/r05/azguide_$v.json 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/r05/azguide_$v.json').read().strip().splitlines()[-1]); print('%-4s %8.2f' % ('$v', d['value']), d['stats']['film_fingerprint'], d['kernel_ms_per_step']['shade'])"
done
