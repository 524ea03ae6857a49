set -o pipefail
for v in lib tw3 tw2; do
  if [ $v = lib ]; then L=cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  HAIRPT_LIB=$PWD/$L timeout -k 10 300 python bench.py --cpu-baseline off --steps 2 --warmup 1 > gpurun_out/tw.log 2>&1 || exit 1
  python -c "
import json; d=json.loads(open('gpurun_out/tw.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['kernel_ms_per_step']['tail'])"
  HAIRPT_LIB=$PWD/$L timeout -k 10 300 python tools/shard_timing.py > gpurun_out/tws.log 2>&1 || exit 1
  grep "^N=8" gpurun_out/tws.log | sed 's/ranks.*->/->/'
done
