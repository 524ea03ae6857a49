# traversal variant A/B: parity + config tests on the default build, then bench with film fingerprints
# usage: scripts/r05/trace_ab.sh [variants...]   (lib is always first)
set -o pipefail
mkdir -p gpurun_out
L0=$PWD/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so
HAIRPT_LIB=$L0 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_configs.py \
  > gpurun_out/trace_ab_tests.log 2>&1 || { echo "TESTS FAIL"; tail -40 gpurun_out/trace_ab_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/trace_ab_tests.log)"
for v in lib "$@"; do
  if [ $v = lib ]; then L=$L0; else L=$PWD/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$L timeout -k 10 300 python bench.py --cpu-baseline off --steps 3 --warmup 1 > gpurun_out/tab_$v.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/tab_$v.log').read().strip().splitlines()[-1]); s=d['stats']
print('%-8s %8.2f' % ('$v', d['value']), d['kernel_ms_per_step'], 'nodes/ray', s['nodes_per_ray'], 'bin', s['binary_nodes_per_ray'], 'fp %.6f' % s['film_fingerprint'])"
done
