# A/B of kernel variant builds (make variant V=<name>): headline bench per build
# usage: scripts/archive/r03_variants.sh name1 name2 ...   ("main" = the default build)
set -o pipefail
mkdir -p gpurun_out/var
for V in "$@"; do
  if [ $V = main ]; then L=""; else L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_$V/libhairpt.so; fi
  HAIRPT_LIB=$L timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/var/$V.json 2> gpurun_out/var/$V.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/var/$V.json').read().strip().splitlines()[-1]); k=d['kernel_ms_per_step']; print('$V', d['value'], d['stats']['film_fingerprint'], 'packet', k['trace_packet'], 'trace', k['trace'], 'shade', k['shade'])"
done
