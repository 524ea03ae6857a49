# load-path occupancy of the traversal kernels: TA busy and the L1 (TCP) stall counters, one
# rocprofv3 --pmc pass per group (TA_BUSY_avr / GRBM_GUI_ACTIVE = fraction of cycles the
# texture-address unit of an average CU is busy)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/tapmc
i=0
for grp in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp \
      -d $ROOT/gpurun_out/tapmc/p$i -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 1 --cpu-baseline off > $ROOT/gpurun_out/tapmc/p$i.log 2>&1) || { echo "PMC FAIL $i"; tail -5 $ROOT/gpurun_out/tapmc/p$i.log; exit 1; }
  python3 $ROOT/tools/pmc_kernel_sums.py $ROOT/gpurun_out/tapmc/p$i k_trace k_shade k_post | tee $ROOT/gpurun_out/tapmc/p$i.txt
  rm -rf $ROOT/gpurun_out/tapmc/p$i
done
