#!/bin/bash
# Round 4: C3 FAST with reciprocal run averages / normalizedWeight (shipped) vs IEEE divisions (wdiv).
set -u
o=gpurun_out/r04s
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_dropin.py -m gpu -x -q -k "wide or consensus or c3" --timeout 300 \
  --timeout-method thread > $o/pytest_wide.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 > $o/c3.json 2> $o/c3.err && \
BCE_LIB=tools/ablate_build/wdiv/libbce_hip.so timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3_wdiv.json 2> $o/c3_wdiv.err && \
timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3_again.json 2> $o/c3_again.err
