#!/bin/bash
# Round 4: tie-break FULL kernel, next array's first batch issued before the output flushes.
set -u
o=gpurun_out/r04aa
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb.json 2> $o/tb.err && \
BCE_LIB=tools/ablate_build/tbnoprebatch/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_noprebatch.json 2> $o/tb_noprebatch.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err
