# round-5 baseline on a fresh box: headline bench (no CPU sample) + one-GPU N=2,4,8 rehearsal
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 2 --cpu-baseline off > gpurun_out/r05/base_bench.json 2> gpurun_out/r05/base_bench.err || exit 1
tail -1 gpurun_out/r05/base_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 400 python3 -u tools/shard_timing.py --all-ranks --reps 3 --ns 8 --balance > gpurun_out/r05/base_reh.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r05/base_reh.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
