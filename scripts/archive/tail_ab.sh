set -o pipefail
for v in lib nosmall; do
  if [ $v = lib ]; then L=cs184-final-project-mitsuba0.5_amd/lib/libhairpt.so; else L=cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so; fi
  echo "== $v"
  HAIRPT_LIB=$PWD/$L timeout -k 10 400 python tools/shard_timing.py > gpurun_out/tab.log 2>&1 || exit 1
  grep "rank 0 kernels" gpurun_out/tab.log | sed 's/.camera.*.tail/ tail/; s/, .gather.*wall/ wall/'
done
