# camera queue sorted by pixel quadrant: the new packet-order test (128 / 256 / 512 spp)
set -o pipefail
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "quadrant or headline" > gpurun_out/r04/qsort_test.log 2>&1 || { tail -40 gpurun_out/r04/qsort_test.log; exit 1; }
tail -6 gpurun_out/r04/qsort_test.log
timeout -k 10 400 python -u tools/shard_timing.py --all-ranks --reps 3 --ns 2,4,8 --balance > gpurun_out/r04/reh_qsort.txt 2>&1 || exit 1
grep "ranks" gpurun_out/r04/reh_qsort.txt | grep -o "N=[0-9] ranks.*" | sed 's/{.*}//'
