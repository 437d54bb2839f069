#!/bin/bash
# Retry a gpurun call on transient (rc=3) failures, at most 4 attempts, 90 s apart.
# Usage: tools/gpu_retry.sh <logfile> <timeout> '<command>'
log=$1; to=$2; cmd=$3
for i in 1 2 3 4; do
  timeout $((to + 900)) /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  rc=$?
  echo "attempt $i rc=$rc" >> "$log.attempts"
  if [ $rc -ne 3 ]; then exit $rc; fi
  sleep 90
done
exit 3
