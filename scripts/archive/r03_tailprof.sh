set -o pipefail
mkdir -p gpurun_out
for v in tp4 tp2; do
for n in 8 1; do
HAIRPT_LIB=$PWD/cs184-final-project-mitsuba0.5_amd/libv_$v/libhairpt.so timeout -k 10 300 python -u tools/tail_profile.py --shards $n > gpurun_out/r03_tailprof_${v}_$n.json 2> gpurun_out/r03_tailprof.err || exit 1
done; done
