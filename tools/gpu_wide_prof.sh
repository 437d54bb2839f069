#!/bin/bash
# GPU box: per-kernel rocprof stats + per-phase stamps of the wide kernel on C3 (fast, exact)
set -u
export TMPDIR=/tmp
o=gpurun_out/wide_prof
mkdir -p $o
for mode in fast exact; do
  BCE_LIB=tools/ablate_build/wide_prof/libbce_hip.so timeout -k 10 200 python3 tools/wide_variants.py one prof --modes $mode \
    > $o/phases_$mode.json 2> $o/phases_$mode.err || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/st_$mode -o run --output-format csv -- \
    python3 tools/wide_variants.py one base --modes $mode > $o/st_$mode.log 2>&1 || exit $?
done
