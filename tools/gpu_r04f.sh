#!/bin/bash
# Round 4: tie-break staging A/B on one box: register batches (shipped) vs single-buffer LDS-DMA.
set -u
o=gpurun_out/r04f
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 \
  --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
BCE_LIB=tools/ablate_build/tbdma1/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb_dma1.json 2> $o/tb_dma1.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err
