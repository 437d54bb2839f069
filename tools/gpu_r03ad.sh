#!/bin/bash
set -u
o=gpurun_out/r03ad
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.txt 2>&1
timeout -k 10 400 python3 tools/wide_variants.py run wbase wnodedup wbase wnodedup --modes fast --reps 20 > $o/ab.txt 2>&1
