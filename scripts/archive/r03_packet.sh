# packet kernel without the inline fallback: overflow parity, packet bit-exactness, headline bench
set -o pipefail
mkdir -p gpurun_out/packet
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_configs.py::test_packet_overflow_launch_is_bit_identical tests/test_gpu_parity.py -k "packet or overflow or tail or smoke or test_render_matches_oracle" > gpurun_out/packet/pytest.log 2>&1 || { tail -30 gpurun_out/packet/pytest.log; exit 1; }
tail -3 gpurun_out/packet/pytest.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-baseline off > gpurun_out/packet/bench.json 2> gpurun_out/packet/bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/packet/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['stats']['film_fingerprint'], d['kernel_ms_per_step'])"
