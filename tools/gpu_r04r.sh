#!/bin/bash
# Round 4: tie-break FULL kernel staging batches: shipped 8/8 vs wr16, pc16+wr16, pc16; tie-break tests.
set -u
o=gpurun_out/r04r
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
for v in tbwr16 tbpc16wr16 tbpc16; do
  BCE_LIB=tools/ablate_build/$v/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb_$v.json 2> $o/tb_$v.err || exit 1
done && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err
