# two-level azimuthal cdf search (variant az2): bit-exactness (BSDF batch, renders), then A/B
set -o pipefail
mkdir -p gpurun_out/az2
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_az2/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_independent_pins.py -m gpu -k "bsdf or marschner or render_matches_oracle or tail or headline" > gpurun_out/az2/pytest.log 2>&1 || { tail -40 gpurun_out/az2/pytest.log; exit 1; }
tail -1 gpurun_out/az2/pytest.log
bash scripts/archive/r03_variants.sh main az2 main az2
