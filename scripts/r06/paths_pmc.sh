#!/bin/bash
# counters of k_paths (HPT_PATHS=1) vs the wavefront kernels: one rocprofv3 --pmc pass per group
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/r06pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  for mode in 1 0; do
    HPT_PATHS=$mode timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp -d $O/g${i}_$mode -o pmc -- \
        python3 $ROOT/bench.py --steps 1 --warmup 2 --cpu-baseline off > $O/g${i}_$mode.log 2>&1 || { echo "group $i mode $mode failed"; tail -3 $O/g${i}_$mode.log; }
    echo "g$i paths=$mode: $(python3 $ROOT/tools/pmc_kernel_sums.py $O/g${i}_$mode k_paths k_trace k_shade k_post k_tail)"
    rm -rf $O/g${i}_$mode
  done
done
