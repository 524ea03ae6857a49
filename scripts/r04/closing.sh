# closing evidence at the final build: the bench line with cpu_baseline against the refreshed traffic file, and the N=8 shard kernel timeline
set -o pipefail
mkdir -p gpurun_out/r04/tlq
timeout -k 10 600 python3 -u bench.py --config furball_marschner --steps 5 --warmup 1 --cpu-spp 96 > gpurun_out/r04/closing_bench.json 2> gpurun_out/r04/closing_bench.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r04/closing_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['traffic'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04/tlq -o tl -- python3 tools/shard_timing.py --reps 3 --ns 8 --balance > gpurun_out/r04/tlq.log 2>&1 || { tail -20 gpurun_out/r04/tlq.log; exit 1; }
find gpurun_out/r04/tlq -name "*kernel_trace.csv" | head -3
