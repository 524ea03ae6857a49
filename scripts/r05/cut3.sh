# eager cut (dry flag polled every 10 us): spill cost with the cut off (poll vs no-poll build), then the
# N=8 rehearsal over cut / tail thresholds, and the launch anatomy of the first one
set -o pipefail
mkdir -p gpurun_out/r05
L=$(pwd)/cs184-final-project-mitsuba0.5_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cut.py > gpurun_out/r05/cut3_pytest.log 2>&1 || { tail -60 gpurun_out/r05/cut3_pytest.log; exit 1; }
tail -1 gpurun_out/r05/cut3_pytest.log
for V in main nopoll; do
  if [ $V = main ]; then LIB=$L/lib/libhairpt.so; else LIB=$L/libv_$V/libhairpt.so; fi
  HAIRPT_LIB=$LIB timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r05/cut3_bench_$V.json 2> gpurun_out/r05/cut3_bench_$V.err || exit 1
  tail -1 gpurun_out/r05/cut3_bench_$V.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V cut off', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['kernel_ms_per_step']['trace'])"
done
for CT in "262144 131072" "262144 524288" "524288 524288" "1048576 524288"; do
  set -- $CT
  HPT_CUT_MIN=$1 HPT_TAIL_PATHS=$2 timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/cut3_reh_$1_$2.txt 2>&1 || exit 1
  echo "cut $1 tail $2: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/cut3_reh_$1_$2.txt) $(grep 'N=8 ranks' gpurun_out/r05/cut3_reh_$1_$2.txt | grep -o 'max.*')"
  grep "N=8 rank 0 kernels" gpurun_out/r05/cut3_reh_$1_$2.txt
done
HPT_TAIL_PATHS=524288 timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/cut3_reh_0_524288.txt 2>&1 || exit 1
echo "cut off tail 524288: $(grep -o '"N1_ms": [0-9.]*' gpurun_out/r05/cut3_reh_0_524288.txt) $(grep 'N=8 ranks' gpurun_out/r05/cut3_reh_0_524288.txt | grep -o 'max.*')"
HPT_CUT_MIN=262144 HAIRPT_LIB=$L/libv_traceprof/libhairpt.so timeout -k 10 300 python -u tools/trace_profile.py --shards 8 > gpurun_out/r05/cut3_prof.jsonl 2> gpurun_out/r05/cut3_prof.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/r05/cut3_prof.jsonl'):
    d = json.loads(l)
    if 'launch' in d: print(d['launch'], d['rays'], 'span', d['span_us'], 'dry', d['dry_at_us'], 'drain', d['drain_us'], 'inflight', d['in_flight_at_dry'])
"
