#!/bin/bash
# the GPU tier + smoke + short bench, then the one-GPU N=2,4,8 rehearsal of the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
bash scripts/r06/gputests.sh && bash scripts/r06/reh.sh "${1:-tier}"
