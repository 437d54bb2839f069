#!/bin/bash
set -u
o=gpurun_out/r03ag
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_wide.txt 2>&1
