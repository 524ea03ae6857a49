# k_tail time split at the N=8 shard (HPT_TAIL_PROFILE variant), then the C4 / C5 one-GPU
# strong-scaling rehearsals at the device-side bounce control build
set -o pipefail
mkdir -p gpurun_out/after
HAIRPT_LIB=$(pwd)/cs184-final-project-mitsuba0.5_amd/libv_tailprof/libhairpt.so timeout -k 10 300 python -u tools/tail_profile.py \
  > gpurun_out/after/tailprof.json 2> gpurun_out/after/tailprof.err || { tail -20 gpurun_out/after/tailprof.err; exit 1; }
cat gpurun_out/after/tailprof.json
bash scripts/archive/r03_rehearsal_c4c5.sh || exit 1
