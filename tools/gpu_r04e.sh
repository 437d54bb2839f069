#!/bin/bash
# Round 4: tie-break lane kernel with two LDS buffers filled by LDS-DMA -- GPU tie-break tests,
# the tb line against the single-buffer build (same box), SQ counters of the new kernel.
set -u
o=gpurun_out/r04e
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak or resolve" --timeout 120 \
  --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb.json 2> $o/tb.err && \
BCE_LIB=tools/ablate_build/tbnodma/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_nodma.json 2> $o/tb_nodma.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err && \
bash tools/gpu_sq.sh tb -- --config tb && cp gpurun_out/sq_tb/summary.txt $o/tb_sq_counters.txt
