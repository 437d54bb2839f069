#!/bin/bash
# Round 4: aggregate_kernel VGPR budget A/B (shipped: compiler choice; aggw6: 6 waves / SIMD).

set -u
o=gpurun_out/r04w
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "aggregat" --timeout 120 --timeout-method thread > $o/pytest_agg.txt 2>&1 && \
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg.json 2> $o/agg.err && \
for v in aggw6; do
  BCE_LIB=tools/ablate_build/$v/libbce_hip.so timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg_$v.json 2> $o/agg_$v.err || exit 1
done && \
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 --no-cpu-baseline > $o/agg_again.json 2> $o/agg_again.err
