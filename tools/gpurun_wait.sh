#!/bin/bash
# run one gpurun call; when no box or slot is free (rc 3, nothing ran, nothing charged) wait and ask again
# usage: tools/gpurun_wait.sh <timeout-s> '<command>'   (log: /tmp/gr.log)
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gr.log 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 90
done
echo "rc=$rc (attempts $i)"
tail -15 /tmp/gr.log
exit $rc
