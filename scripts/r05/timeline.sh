# rocprofv3 kernel trace of one N=8 shard frame at the final build, summarised per launch
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=r05 N=8 bash $ROOT/scripts/gpu_timeline.sh || exit 1
DB=$(dirname $(find $ROOT/gpurun_out/timeline_r05/db -name "*.db" | head -1))
python3 $ROOT/tools/launch_timeline.py --summarize $DB > $ROOT/gpurun_out/timeline_r05/r05_timeline_n8.md || exit 1
rm -rf $ROOT/gpurun_out/timeline_r05/db
tail -3 $ROOT/gpurun_out/timeline_r05/r05_timeline_n8.md
