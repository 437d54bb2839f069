#!/bin/bash
# Round 4: agg rocprof stats + PMC of the line's own launches (no median phase).
set -u
export TMPDIR=/tmp
bash tools/gpu_profile.sh agg aggregate_kernel groups=10000 -- --config agg --single-mode
