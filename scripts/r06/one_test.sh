#!/bin/bash
# one GPU test file (or node id) with the standard limits: scripts/r06/one_test.sh tests/x.py[::name]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/r06/one_test.log 2>&1
rc=$?
tail -15 gpurun_out/r06/one_test.log
exit $rc
