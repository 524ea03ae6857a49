# resumable cut with the resumed rays spread over every cursor shard: tests, bench, N=8 rehearsal,
# and the N=8 launch anatomy (traceprof variant) cut off / on
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r05/cut2_pytest.log 2>&1 || { tail -60 gpurun_out/r05/cut2_pytest.log; exit 1; }
tail -1 gpurun_out/r05/cut2_pytest.log
for C in 0 262144; do
  HPT_CUT_MIN=$C timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r05/cut2_bench_$C.json 2> gpurun_out/r05/cut2_bench_$C.err || exit 1
  tail -1 gpurun_out/r05/cut2_bench_$C.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cut_min $C', d['value'], d['ms_per_step'], d['stats']['film_fingerprint'], d['stats'].get('cut_rays_per_step'), d['kernel_ms_per_step'])"
  HPT_CUT_MIN=$C timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/cut2_reh_$C.txt 2>&1 || exit 1
  echo "cut_min $C: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/cut2_reh_$C.txt) $(grep 'N=8 ranks' gpurun_out/r05/cut2_reh_$C.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r05/cut2_reh_$C.txt
  HPT_CUT_MIN=$C HAIRPT_LIB=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_traceprof/libhairpt.so timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/r05/cut2_prof_$C.jsonl 2> gpurun_out/r05/cut2_prof_$C.err || exit 1
  python3 -c "
import json
for l in open('gpurun_out/r05/cut2_prof_$C.jsonl'):
    d = json.loads(l)
    if 'launch' in d: print(d['launch'], d['rays'], 'span', d['span_us'], 'dry', d['dry_at_us'], 'drain', d['drain_us'], 'inflight', d['in_flight_at_dry'])
"
done
