#!/bin/bash
# Round 4: C2 headline with 4-wave workgroups (one wave per SIMD, no VGPR spills) vs 8.
set -u
o=gpurun_out/r04ab
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $o/c2.json 2> $o/c2.err && \
BCE_LIB=tools/ablate_build/tab4w/libbce_hip.so timeout -k 10 300 python3 bench.py --no-secondary > $o/c2_tab4w.json 2> $o/c2_tab4w.err && \
timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline > $o/c2_again.json 2> $o/c2_again.err
