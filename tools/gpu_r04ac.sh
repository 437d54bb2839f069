#!/bin/bash
# Round 4: tie-break round() edge cases on FULL tiles.
set -u
o=gpurun_out/r04ac
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 --timeout-method thread > $o/pytest_tb.txt 2>&1
