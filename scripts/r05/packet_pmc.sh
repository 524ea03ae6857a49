# scalar / vector instruction counts of the packet pass per build (one rocprofv3 --pmc pass each)
# usage: scripts/r05/packet_pmc.sh v1 v2 ...   (lib is always first)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out/pkpmc
for v in lib "$@"; do
  if [ $v = lib ]; then L=$ROOT/cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=$ROOT/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  (cd /tmp && export TMPDIR=/tmp && HAIRPT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAVES \
      -d $ROOT/gpurun_out/pkpmc/$v -o pmc -- python3 $ROOT/bench.py --steps 1 --warmup 1 --cpu-baseline off > $ROOT/gpurun_out/pkpmc/$v.log 2>&1) || { echo "PMC FAIL $v"; tail -5 $ROOT/gpurun_out/pkpmc/$v.log; exit 1; }
  echo "$v: $(python3 $ROOT/tools/pmc_kernel_sums.py $ROOT/gpurun_out/pkpmc/$v ${PMC_KERNELS:-k_trace_packet})"
  rm -rf $ROOT/gpurun_out/pkpmc/$v
done
