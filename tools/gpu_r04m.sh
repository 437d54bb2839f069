#!/bin/bash
# Round 4: tie-break rocprof stats + PMC for the FULL kernel alone (the second launch shares
# the name prefix and would halve the per-launch average).
set -u
export TMPDIR=/tmp
bash tools/gpu_profile.sh tb "tiebreak_lpm_kernel<true, false, 1>" markets=1000000 -- --config tb
