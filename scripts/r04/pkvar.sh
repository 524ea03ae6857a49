# packet-kernel leaf batch with quadrant packets: 1 / 2 (shipped) / 4 records per round trip
set -o pipefail
mkdir -p gpurun_out/r04
for v in lb1 lb4; do
  HAIRPT_LIB=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --cpu-baseline off > gpurun_out/r04/pkvar_$v.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r04/pkvar_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['kernel_ms_per_step']['trace_packet'], d['stats']['film_fingerprint'])"
done
