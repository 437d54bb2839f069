#!/bin/bash
# Round 4: tie-break with the touch prefetch off -- tests, bench line, rocprof stats + PMC.
set -u
o=gpurun_out/r04n
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 \
  --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb.json 2> $o/tb.err && \
bash tools/gpu_profile.sh tb "tiebreak_lpm_kernel<true, false, 1>" markets=1000000 -- --config tb
