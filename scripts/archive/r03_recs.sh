# queue-ordered path records (shade / post / shadow records): the full GPU tier, then the bench
set -o pipefail
mkdir -p gpurun_out/recs
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/recs/gputests.log 2>&1 || { tail -40 gpurun_out/recs/gputests.log; exit 1; }
tail -1 gpurun_out/recs/gputests.log
bash scripts/archive/r03_variants.sh main main || exit 1
python -c "import json; d=json.loads(open('gpurun_out/var/main.json').read().strip().splitlines()[-1]); print(d['kernel_ms_per_step'])"
