#!/bin/bash
# Chain GPU steps on the box; stop at the first crash / timeout / GPU fault.
# Usage: tools/gpu_run.sh "<step1>" "<step2>" ...   (each step gets its own timeout prefix)
# pytest exit 1 (= failing tests, not a crash) does not stop the chain; anything else does.
set -u
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i+1))
  echo "=== step $i: $step" | tee -a gpurun_out/steps.log
  bash -c "$step"
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
