# k_tail with the one-round-trip Sobol look-up: tail bit-identity tests on the variant, per-kernel A/B,
# and the N=8 rehearsal on both builds
set -o pipefail
mkdir -p gpurun_out/r05
V=$PWD/cs184-final-project-mitsuba0.5_amd/libv_${1:-sr}/libhairpt.so
HAIRPT_LIB=$V timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "tail or sobol" > gpurun_out/r05/tailrows_tests.log 2>&1 || { tail -30 gpurun_out/r05/tailrows_tests.log; exit 1; }
tail -1 gpurun_out/r05/tailrows_tests.log
bash scripts/kernel_ab.sh ${1:-sr} || exit 1
for L in lib ${1:-sr}; do
  if [ $L = lib ]; then LL=$PWD/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else LL=$V; fi
  HAIRPT_LIB=$LL timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/tailrows_reh_$L.txt 2>&1 || exit 1
  echo "$L: $(grep 'N=8 ranks' gpurun_out/r05/tailrows_reh_$L.txt | grep -o 'max.*')  $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/tailrows_reh_$L.txt)"
done
