# FETCH_SIZE / WRITE_SIZE calibration on known-byte gathers, streams and scatters (tools/fetch_calib.hip)
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/fcal
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o f -- "$ROOT/tools/fetch_calib" > "$OUT/run.log" 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o w -- "$ROOT/tools/fetch_calib" > "$OUT/run_w.log" 2>&1 || exit 1
