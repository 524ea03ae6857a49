#!/bin/bash
# instruction-cache counters of k_paths vs the wavefront kernels (one --pmc pass each)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r06pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQC_TC_INST[A-Z_]*" $O/avail.txt | sort -u | tr '\n' ' '; echo
CTR=$(grep -o "SQC_ICACHE_MISSES\b\|SQC_ICACHE_HITS\b\|SQ_IFETCH\b" $O/avail.txt | sort -u | tr '\n' ' ')
echo "counters: $CTR"
[ -n "$CTR" ] || exit 0
for mode in 1 0; do
  HPT_PATHS=$mode timeout -k 10 200 rocprofv3 --kernel-trace --pmc $CTR -d $O/ic_$mode -o pmc -- \
      python3 $ROOT/bench.py --steps 1 --warmup 2 --cpu-baseline off > $O/ic_$mode.log 2>&1 || { echo "mode $mode failed"; tail -3 $O/ic_$mode.log; }
  echo "paths=$mode: $(python3 $ROOT/tools/pmc_kernel_sums.py $O/ic_$mode k_paths k_trace k_shade k_post)"
  rm -rf $O/ic_$mode
done
