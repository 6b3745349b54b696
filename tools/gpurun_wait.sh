#!/bin/bash
# Submit one gpurun call; while the pool has no box (exit 3: nothing ran, nothing charged) wait and
# submit again, up to ~25 minutes.  Any other exit code (the command ran) is returned as is.
# usage: tools/gpurun_wait.sh <timeout_s> '<command>'
T=$1; shift
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 75
done
exit 3
