#!/bin/bash
# Round 4: refresh the f4 line and its rocprof stats + PMC after the VGPR-budget change.
set -u
o=gpurun_out/r04x
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg.json 2> $o/agg.err && \
bash tools/gpu_profile.sh agg aggregate_kernel groups=10000 -- --config agg --single-mode
