# k_post reads its continuation's bsdf weight / throughput / state from a queue-ordered record
# written by k_shade: render parity tests, then the bench (kernel times per step)
set -o pipefail
mkdir -p gpurun_out/postrec
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "render or tail or headline or full_size or multi" > gpurun_out/postrec/pytest.log 2>&1 || { tail -40 gpurun_out/postrec/pytest.log; exit 1; }
tail -1 gpurun_out/postrec/pytest.log
bash scripts/archive/r03_variants.sh main main || exit 1
python -c "import json; d=json.loads(open('gpurun_out/var/main.json').read().strip().splitlines()[-1]); print(d['kernel_ms_per_step'])"
