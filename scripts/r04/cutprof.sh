# k_trace launch anatomy with the launch cut on / off at the N=8 shard (traceprof variant: per-wave dry / exit times)
set -o pipefail
mkdir -p gpurun_out/r04
L=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_traceprof/libhairpt.so
for C in 0 1; do
  HPT_CUT=$C HAIRPT_LIB=$L timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/r04/cutprof_c$C.jsonl 2> gpurun_out/r04/cutprof_c$C.err || exit 1
  echo "cut=$C"; python3 -c "
import json
for l in open('gpurun_out/r04/cutprof_c$C.jsonl'):
    d = json.loads(l)
    if 'launch' in d: print(d['launch'], d['rays'], 'span', d['span_us'], 'dry', d['dry_at_us'], 'drain', d['drain_us'], 'inflight', d['in_flight_at_dry'], 'alive', d.get('waves_alive_after_dry_us'))
"
done
