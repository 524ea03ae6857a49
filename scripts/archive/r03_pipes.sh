# Interleaved wavefront pipelines (HPT_PIPES) with stream priorities (HPT_PIPE_PRIO) and splits
# (HPT_PIPE_SPLIT): headline fingerprint + one-GPU N=8 rehearsal per setting
set -o pipefail
mkdir -p gpurun_out/pipes
run() { # tag env...
  tag=$1; shift
  echo "== $tag"
  env "$@" timeout -k 10 300 python -u tools/shard_timing.py --reps 2 --ns 8 > gpurun_out/pipes/shards_$tag.log 2>&1 || exit 1
  grep "^N=8 ranks\|N1_ms" gpurun_out/pipes/shards_$tag.log | cut -c1-200
}
run base HPT_PIPES=1
run p2prio HPT_PIPES=2 HPT_PIPE_PRIO=1
run p2prio70 HPT_PIPES=2 HPT_PIPE_PRIO=1 HPT_PIPE_SPLIT=0.7
run p2prio85 HPT_PIPES=2 HPT_PIPE_PRIO=1 HPT_PIPE_SPLIT=0.85
run p2noprio70 HPT_PIPES=2 HPT_PIPE_SPLIT=0.7
HPT_PIPES=2 HPT_PIPE_PRIO=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-baseline off > gpurun_out/pipes/bench_p2prio.json 2> gpurun_out/pipes/bench_p2prio.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/pipes/bench_p2prio.json').read().strip().splitlines()[-1]); print(d['value'], d['stats']['film_fingerprint'])"
