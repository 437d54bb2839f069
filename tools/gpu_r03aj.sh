#!/bin/bash
# LDS-DMA helpers that save/restore M0 (variant wm0save, tools/wide_variants.py): pipe-kernel
# parity (S > 2^18 tables) and the C2 line at S = 1M / 12k with that build.
set -u
o=gpurun_out/r03aj
mkdir -p $o
export BCE_LIB=tools/ablate_build/wm0save/libbce_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_consensus.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --no-secondary --sources 1000000 --steps 30 --warmup 5 > $o/c2_S1000000.json 2> $o/c2_S1000000.err && \
timeout -k 10 200 python3 bench.py --no-secondary --sources 12000 --steps 30 --warmup 5 > $o/c2_S12000.json 2> $o/c2_S12000.err
