#!/bin/bash
# Headline profile with the PMC limiter evidence: rocprofv3 kernel trace, FETCH_SIZE / WRITE_SIZE
# passes, the occupancy / stall / cache counter groups (scripts/gpu_pmc.sh), the summary with
# --pmc (-> profiles/r04_furball_marschner_kernels.md + traffic JSON with `limiter`), then the
# bench line with the 10-30 s CPU sample.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cfg=furball_marschner
OUT=$ROOT/gpurun_out/cfg/prof_$cfg
mkdir -p "$OUT"
run() { (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 "$@" -o bench -- \
      python3 "$ROOT/bench.py" --config $cfg --steps 5 --warmup 1 --cpu-baseline off) ; }
echo "== trace"; run --kernel-trace --stats -d "$OUT/trace" > "$OUT/bench_trace.log" 2>&1 || exit 1
echo "== fetch"; run --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" > "$OUT/bench_fetch.log" 2>&1 || exit 1
echo "== write"; run --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" > "$OUT/bench_write.log" 2>&1 || exit 1
echo "== pmc groups"; bash "$ROOT/scripts/gpu_pmc.sh" r04 --config $cfg --steps 2 --warmup 1 || exit 1
WL=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/bench_trace.log') if l.startswith('{\"metric\"')][-1]['config']['workload'])") || exit 1
python3 "$ROOT/tools/rocpd_summary.py" "$OUT" --pmc "$ROOT/gpurun_out/pmc_r04" --out "$ROOT/gpurun_out/cfg/r04_${cfg}_kernels.md" \
    --title "r04 $cfg: rocprofv3 summary of bench.py --config $cfg --steps 5 --warmup 1 (PMC groups: --steps 2)" \
    --json "$ROOT/gpurun_out/cfg/traffic_${cfg}.json" --workload "$WL" > /dev/null || exit 1
cp "$ROOT/gpurun_out/cfg/traffic_${cfg}.json" "$ROOT/gpurun_out/cfg/r04_traffic_${cfg}.json" || exit 1
echo "== bench with cpu_baseline"
timeout -k 10 600 python3 -u "$ROOT/bench.py" --config $cfg --steps 5 --warmup 1 --cpu-spp 96 > "$ROOT/gpurun_out/cfg/r04_bench_${cfg}.json" \
    2> "$ROOT/gpurun_out/cfg/r04_bench_${cfg}.err" || exit 1
python3 -c "import json; d=json.loads(open('$ROOT/gpurun_out/cfg/r04_bench_${cfg}.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['roofline']['limiter'])"
