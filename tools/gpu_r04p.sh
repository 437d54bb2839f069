#!/bin/bash
# Round 4: tie-break general body rebuilt (bit-set validity / run masks, fast round, reciprocal means): ragged + uniform lines, all tie-break tests.

set -u
o=gpurun_out/r04p
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --ragged --steps 20 --warmup 3 > $o/tb_ragged.json 2> $o/tb_ragged.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o tb -- python3 bench.py --config tb --ragged --steps 10 --warmup 2 --no-cpu-baseline > $o/prof.log 2>&1
