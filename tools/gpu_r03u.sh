#!/bin/bash
# GPU box, repo root: wide parity, wide A/B (flip-31 stage, 1-wave HR), C3 shard steps with and
# without the small-bin stream alternation, C4 line.  Stops at the first failing step.
set -u
o=gpurun_out/r03u
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_wide.txt 2>&1 && \
timeout -k 10 400 python3 tools/wide_variants.py run wbase wnoflip31 whr2nw1 wxwsel wntst wbase wnoflip31 whr2nw1 wxwsel wntst --modes fast --reps 20 > $o/ab.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/shards_alt.json 2> $o/shards_alt.err && \
BCE_LIB=tools/ablate_build/wnoalt/libbce_hip.so timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/shards_noalt.json 2> $o/shards_noalt.err && \
timeout -k 10 200 python3 bench.py --config c4 --steps 200 --warmup 20 > $o/c4.json 2> $o/c4.err
