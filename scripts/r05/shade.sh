# k_shade register/LDS variants: BSDF parity on the shipped build, then per-kernel A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bsdf or marschner" tests/test_independent_pins.py > gpurun_out/shade_tests.log 2>&1 || { tail -30 gpurun_out/shade_tests.log; exit 1; }
tail -3 gpurun_out/shade_tests.log
bash scripts/kernel_ab.sh "$@"
