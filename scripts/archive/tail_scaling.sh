#!/bin/bash
# N=8 rank timings (one-GPU rehearsal) for several k_tail thresholds (HPT_TAIL_PATHS)
set -o pipefail
mkdir -p gpurun_out/tailscale
for t in ${THRESHOLDS:-131072 262144 524288 1048576}; do
  HPT_TAIL_PATHS=$t timeout -k 10 300 python3 tools/shard_timing.py > gpurun_out/tailscale/t$t.json 2> gpurun_out/tailscale/t$t.err || { echo "fail $t"; exit 1; }
  echo "tail $t: $(grep -E 'N=8 ranks|N=1' gpurun_out/tailscale/t$t.err | tail -1 | cut -c1-200)"
  python3 -c "import json;d=json.load(open('gpurun_out/tailscale/t$t.json'));print('  N1 %.2f ms, N8 max %.2f ms, eff %.3f' % (d['N1_ms'], d['shards']['8']['max_ms'], d['shards']['8']['efficiency']))"
done
