# packet-pass variants: packet bit-exactness tests on each build, then per-kernel A/B
# usage: scripts/r05/packet.sh v1 v2 ...   (lib is always first)
set -o pipefail
mkdir -p gpurun_out
for v in lib "$@"; do
  if [ $v = lib ]; then L=$PWD/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=$PWD/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -k "packet_trace_bit_exact or camera_quadrant or trace_bit_exact" tests/test_gpu_configs.py::test_packet_overflow_launch_is_bit_identical \
    > gpurun_out/packet_tests_$v.log 2>&1 || { echo "TESTS FAIL $v"; tail -30 gpurun_out/packet_tests_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/packet_tests_$v.log)"
done
bash scripts/kernel_ab.sh "$@"
