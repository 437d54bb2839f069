#!/bin/bash
# GPU box, repo root: GPU suite, default bench (with secondary lines), C2 source-count sweep
# on HEAD (hybrid LDS/global table), compact-mode C2.  Stops at the first failing step.
set -u
o=gpurun_out/r03h
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > $o/default.json 2> $o/default.err && \
for S in 12000 20000 50000 100000 262144 1000000; do
  timeout -k 10 200 python3 bench.py --no-secondary --sources $S --steps 30 --warmup 5 > $o/c2_S$S.json 2> $o/c2_S$S.err || exit 1
done && \
timeout -k 10 200 python3 bench.py --no-secondary --compact > $o/c2_compact.json 2> $o/c2_compact.err
