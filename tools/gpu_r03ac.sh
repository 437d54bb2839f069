#!/bin/bash
set -u
o=gpurun_out/r03ac
mkdir -p $o
BCE_LIB=tools/ablate_build/w5split/libbce_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_w5.txt 2>&1 && \
timeout -k 10 400 python3 tools/wide_variants.py run wbase w5split wbase w5split --modes fast --reps 20 > $o/ab.txt 2>&1
