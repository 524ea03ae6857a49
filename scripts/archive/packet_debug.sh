set -o pipefail
for v in bin lib; do
  if [ $v = lib ]; then L=cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  echo "== $v"
  HAIRPT_LIB=$PWD/$L timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "packet_trace or trace_bit_exact" -q --timeout 150 --timeout-method thread 2>&1 | grep -E "passed|failed|Mismatched|^FAILED" | head -12
done
