# two-level packet traversal: bit-exactness tests, then A/B against the binary packet build
set -o pipefail
mkdir -p gpurun_out/pk4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py::test_packet_overflow_launch_is_bit_identical tests/test_gpu_parity.py -k "packet or overflow or test_render_matches_oracle" > gpurun_out/pk4/pytest.log 2>&1 || { tail -40 gpurun_out/pk4/pytest.log; exit 1; }
tail -3 gpurun_out/pk4/pytest.log
bash scripts/archive/r03_variants.sh main pkbin main pkbin
