# three-level kd nodes (variant n8): bit-exactness through the variant, then A/B bench
set -o pipefail
mkdir -p gpurun_out/n8
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_n8/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "trace_bit_exact or render_matches_oracle or tail or packet or independent" > gpurun_out/n8/pytest.log 2>&1 || { tail -40 gpurun_out/n8/pytest.log; exit 1; }
tail -3 gpurun_out/n8/pytest.log
bash scripts/archive/r03_variants.sh main n8 main n8
