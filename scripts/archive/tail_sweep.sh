set -o pipefail
for t in 131072 1000000 2200000 5000000; do
  HPT_TAIL_PATHS=$t timeout -k 10 300 python tools/shard_timing.py > gpurun_out/tail_$t.log 2>&1 || { echo FAIL $t; exit 1; }
  echo "tail $t"; grep "^N=" gpurun_out/tail_$t.log | sed 's/ranks//'
done
