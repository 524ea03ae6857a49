# Final per-config bench lines (roofline from the committed traffic JSONs + cpu_baseline with a
# ~10-30 s CPU sample): C2 straight_kk, C3 furball_marschner, C4 curly_marschner, C5 furball_1m
set -o pipefail
mkdir -p gpurun_out/lines
line() { # config steps cpu-spp
  echo "== $1"
  timeout -k 10 900 python3 -u bench.py --config $1 --steps $2 --warmup 1 --cpu-spp $3 > gpurun_out/lines/r03_bench_$1.json 2> gpurun_out/lines/r03_bench_$1.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/lines/r03_bench_$1.json').read().strip().splitlines()[-1]); c=d['cpu_baseline']; print(d['value'], d['roofline']['frac'], c['value'], c['cores'], (c['cpu_share'] or {}).get('value'), c['sample'][:70])"
}
line straight_kk 10 64
line furball_marschner 5 96
line curly_marschner 2 32
line furball_1m 2 24
