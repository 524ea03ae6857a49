# packet traversal with both children fetched before the decision (variant pkpf): bit-exactness, A/B
set -o pipefail
mkdir -p gpurun_out/pkpf
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_pkpf/libhairpt.so
HAIRPT_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "packet or trace_bit_exact" > gpurun_out/pkpf/pytest.log 2>&1 || { tail -40 gpurun_out/pkpf/pytest.log; exit 1; }
tail -1 gpurun_out/pkpf/pytest.log
bash scripts/archive/r03_variants.sh main pkpf main pkpf
