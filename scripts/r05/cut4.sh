# lazy cut before Russian roulette only, k_tail taking the trailing paths (HPT_CUT_TAIL): tests, then
# the N=8 rehearsal and the headline frame over the tail threshold, and the launch anatomy
set -o pipefail
mkdir -p gpurun_out/r05
L=$(pwd)/cs184-final-project-mitsuba0.5_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r05/cut4_pytest.log 2>&1 || { tail -60 gpurun_out/r05/cut4_pytest.log; exit 1; }
tail -1 gpurun_out/r05/cut4_pytest.log
for CT in "0 131072" "262144 262144" "262144 524288" "262144 1048576"; do
  set -- $CT
  HPT_CUT_MIN=$1 HPT_CUT_TAIL=$2 timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/cut4_reh_$1_$2.txt 2>&1 || exit 1
  echo "cut $1 tail $2: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/cut4_reh_$1_$2.txt) $(grep 'N=8 ranks' gpurun_out/r05/cut4_reh_$1_$2.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r05/cut4_reh_$1_$2.txt
done
HPT_CUT_MIN=262144 HAIRPT_LIB=$L/libv_traceprof/libhairpt.so timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/r05/cut4_prof.jsonl 2> gpurun_out/r05/cut4_prof.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/r05/cut4_prof.jsonl'):
    d = json.loads(l)
    if 'launch' in d: print(d['launch'], d['rays'], 'span', d['span_us'], 'dry', d['dry_at_us'], 'drain', d['drain_us'], 'inflight', d['in_flight_at_dry'])
"
