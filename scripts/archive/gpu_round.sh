#!/bin/bash
# One GPU call of the build/measure loop (run on the box from the repo root through gpurun):
#   1. the gpu-marked tests (parity, configs)
#   2. the headline bench with the default library, then with every libv_<V> variant named in $VARIANTS
# Usage: TAG=r02a VARIANTS="w4" scripts/archive/gpu_round.sh [pytest selection]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
SEL=${1:-tests}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread \
      > $OUT/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --cpu-baseline ${CPU:-off} > $OUT/bench.log 2>&1 \
    || { echo "bench failed rc=$?"; tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
for v in $VARIANTS; do
  HAIRPT_LIB=$ROOT/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so timeout -k 10 300 \
      python bench.py --steps ${STEPS:-10} --warmup 2 --cpu-baseline off > $OUT/bench_$v.log 2>&1 \
      || { echo "bench $v failed rc=$?"; tail -20 $OUT/bench_$v.log; exit 1; }
  echo "== $v"; tail -1 $OUT/bench_$v.log | cut -c1-400
done
