# One frame of every bench config on one GPU (DESIGN.md "Other configs")
set -o pipefail
mkdir -p gpurun_out
for c in straight_kk furball_roughplastic haircurl_roughplastic curly_marschner furball_1m; do
  timeout -k 10 400 python bench.py --config $c --cpu-baseline off --steps 1 --warmup 1 > gpurun_out/cfg_$c.log 2>&1 || { echo "FAIL $c"; tail -3 gpurun_out/cfg_$c.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/cfg_$c.log').read().strip().splitlines()[-1]); print('%-24s %8.2f Mpaths/s %9.2f ms/frame prepare %.2f s' % ('$c', d['value'], d['ms_per_step'], d['config']['prepare_s']), d['config']['workload'])"
done
