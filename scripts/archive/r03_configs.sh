#!/bin/bash
# Round-3 per-config measurement on the GPU box (gpurun from the repo root):
# for each config, a rocprofv3 kernel trace + stats, the FETCH_SIZE and WRITE_SIZE PMC passes,
# a committed-style summary (tools/rocpd_summary.py -> profiles/), then the bench line with
# roofline + cpu_baseline (which reads the traffic JSON just written).
# Usage: scripts/archive/r03_configs.sh <config> [<config> ...]
#   C2 straight_kk, C3 furball_marschner (headline), C4 curly_marschner, C5 furball_1m
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/cfg"
for cfg in "$@"; do
  case $cfg in
    furball_1m|curly_marschner) CPU="--cpu-spp 1" ; STEPS="--steps 2 --warmup 1" ;;
    *) CPU="--cpu-spp 24" ; STEPS="--steps 5 --warmup 1" ;;
  esac
  OUT=$ROOT/gpurun_out/cfg/prof_$cfg
  mkdir -p "$OUT"
  echo "== $cfg: kernel trace"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o bench -- \
      python3 "$ROOT/bench.py" --config $cfg $STEPS --cpu-baseline off > "$OUT/bench_trace.log" 2>&1) || exit 1
  echo "== $cfg: FETCH_SIZE"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o bench -- \
      python3 "$ROOT/bench.py" --config $cfg $STEPS --cpu-baseline off > "$OUT/bench_fetch.log" 2>&1) || exit 1
  echo "== $cfg: WRITE_SIZE"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o bench -- \
      python3 "$ROOT/bench.py" --config $cfg $STEPS --cpu-baseline off > "$OUT/bench_write.log" 2>&1) || exit 1
  WL=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/bench_trace.log') if l.startswith('{\"metric\"')][-1]['config']['workload'])") || exit 1
  python3 "$ROOT/tools/rocpd_summary.py" "$OUT" --out "$ROOT/gpurun_out/cfg/r03_${cfg}_kernels.md" \
      --title "r03 $cfg: rocprofv3 summary of bench.py --config $cfg $STEPS" \
      --json "$ROOT/gpurun_out/cfg/traffic_${cfg}.json" --workload "$WL" > /dev/null || exit 1
  cp "$ROOT/gpurun_out/cfg/traffic_${cfg}.json" "$ROOT/profiles/traffic_${cfg}.json" || exit 1
  echo "== $cfg: bench with cpu_baseline"
  timeout -k 10 600 python3 -u "$ROOT/bench.py" --config $cfg $STEPS $CPU > "$ROOT/gpurun_out/cfg/r03_bench_${cfg}.json" \
      2> "$ROOT/gpurun_out/cfg/r03_bench_${cfg}.err" || exit 1
  tail -c 400 "$ROOT/gpurun_out/cfg/r03_bench_${cfg}.json"; echo
done
echo "configs done"
