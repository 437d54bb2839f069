#!/bin/bash
# GPU box, repo root: wide/consensus parity on the shipped build, then C3 FAST SQ counters.
set -u
o=gpurun_out/r03v
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_wide.txt 2>&1 && \
bash tools/gpu_sq.sh c3fast -- --config c3 --mode fast
