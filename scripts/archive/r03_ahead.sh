# device-side bounce control: bit-identity tests, then the one-GPU strong-scaling rehearsal
# with the host loop (HPT_BOUNCE_AHEAD=0) and with bounces launched ahead, then bench.py
set -o pipefail
mkdir -p gpurun_out/ahead
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bounce_ahead.py \
  "tests/test_gpu_parity.py::test_tail_kernel_bit_identical" > gpurun_out/ahead/pytest.log 2>&1 || { tail -40 gpurun_out/ahead/pytest.log; exit 1; }
tail -2 gpurun_out/ahead/pytest.log
for a in 0 1; do
  HPT_BOUNCE_AHEAD=$a timeout -k 10 300 python -u tools/shard_timing.py --all-ranks > gpurun_out/ahead/shards_$a.log 2>&1 || { tail -20 gpurun_out/ahead/shards_$a.log; exit 1; }
  echo "ahead=$a"; grep -E "ranks|rank 0 kernels" gpurun_out/ahead/shards_$a.log | sed 's/ranks {.*} ->/ ->/' | cut -c1-220
done
timeout -k 10 600 python -u bench.py > gpurun_out/ahead/bench.json 2> gpurun_out/ahead/bench.err || { tail -20 gpurun_out/ahead/bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/ahead/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stats'].get('film_fingerprint'))"
