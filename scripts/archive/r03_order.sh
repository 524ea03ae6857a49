# camera packets in cost order: bit-identity tests, then the one-GPU strong-scaling rehearsal with the
# block-order queue (HPT_PACKET_ORDER=0) and the cost-ordered queue, then bench.py
set -o pipefail
mkdir -p gpurun_out/order
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bounce_ahead.py \
  > gpurun_out/order/pytest.log 2>&1 || { tail -40 gpurun_out/order/pytest.log; exit 1; }
tail -2 gpurun_out/order/pytest.log
for a in 0 1; do
  HPT_PACKET_ORDER=$a timeout -k 10 300 python -u tools/shard_timing.py --all-ranks > gpurun_out/order/shards_$a.log 2>&1 || { tail -20 gpurun_out/order/shards_$a.log; exit 1; }
  echo "order=$a"; grep -E "ranks|rank 0 kernels" gpurun_out/order/shards_$a.log | sed 's/ranks {.*} ->/ ->/' | cut -c1-220
done
timeout -k 10 600 python -u bench.py > gpurun_out/order/bench.json 2> gpurun_out/order/bench.err || { tail -20 gpurun_out/order/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/order/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stats'].get('film_fingerprint'))"
