#!/bin/bash
# Per-config refresh at the round-6 build: rocprofv3 kernel trace + stats, FETCH_SIZE / WRITE_SIZE
# passes, the summary and traffic JSON (tools/rocpd_summary.py), then the bench line with roofline
# (reading that traffic JSON) and the CPU sample.
# Usage: scripts/r06/configs.sh "<config>:<steps>:<cpu-spp>" ...  [PMC=1: also the PMC groups]
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/gpurun_out/r06cfg"
for spec in "$@"; do
  IFS=: read cfg steps cspp <<< "$spec"
  OUT=$ROOT/gpurun_out/r06cfg/prof_$cfg
  mkdir -p "$OUT"
  run() { (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 "$@" -o bench -- \
        python3 "$ROOT/bench.py" --config $cfg --steps $steps --warmup 1 --cpu-baseline off) ; }
  echo "== $cfg trace"; run --kernel-trace --stats -d "$OUT/trace" > "$OUT/bench_trace.log" 2>&1 || exit 1
  echo "== $cfg fetch"; run --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" > "$OUT/bench_fetch.log" 2>&1 || exit 1
  echo "== $cfg write"; run --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" > "$OUT/bench_write.log" 2>&1 || exit 1
  PMCARG=
  if [ "${PMC:-0}" = 1 ]; then
    echo "== $cfg pmc groups"; bash "$ROOT/scripts/gpu_pmc.sh" r06_$cfg --config $cfg --steps 2 --warmup 1 || exit 1
    PMCARG="--pmc $ROOT/gpurun_out/pmc_r06_$cfg"
  fi
  WL=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/bench_trace.log') if l.startswith('{\"metric\"')][-1]['config']['workload'])") || exit 1
  python3 "$ROOT/tools/rocpd_summary.py" "$OUT" $PMCARG --out "$ROOT/gpurun_out/r06cfg/r06_${cfg}_kernels.md" \
      --title "r06 $cfg: rocprofv3 summary of bench.py --config $cfg --steps $steps --warmup 1" \
      --json "$ROOT/profiles/traffic_${cfg}.json" --workload "$WL" > /dev/null || exit 1
  cp "$ROOT/profiles/traffic_${cfg}.json" "$ROOT/gpurun_out/r06cfg/traffic_${cfg}.json" || exit 1
  # the databases stay on the box (gpurun merges at most 64 MiB back): the summary has what is kept
  rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write" "$ROOT/gpurun_out/pmc_r06_$cfg"
  echo "== $cfg bench with cpu_baseline"
  timeout -k 10 600 python3 -u "$ROOT/bench.py" --config $cfg --steps $steps --warmup 1 --cpu-spp $cspp \
      > "$ROOT/gpurun_out/r06cfg/r06_bench_${cfg}.json" 2> "$ROOT/gpurun_out/r06cfg/r06_bench_${cfg}.err" || exit 1
  python3 -c "import json; d=json.loads(open('$ROOT/gpurun_out/r06cfg/r06_bench_${cfg}.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print('$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['frac_hbm'], c['value'], c['cores'])"
done
