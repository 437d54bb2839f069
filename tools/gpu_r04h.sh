#!/bin/bash
# Round 4: tie-break FULL-tile kernel (PART 1 + PART 2 launches) vs one general launch (tbnofull).
set -u
o=gpurun_out/r04h
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q -k "tiebreak" --timeout 120 \
  --timeout-method thread > $o/pytest_tb.txt 2>&1 && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb.json 2> $o/tb.err && \
BCE_LIB=tools/ablate_build/tbnofull/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_nofull.json 2> $o/tb_nofull.err && \
BCE_LIB=tools/ablate_build/tbkvsort/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_kvsort.json 2> $o/tb_kvsort.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o tb -- python3 bench.py --config tb --steps 10 --warmup 2 --no-cpu-baseline > $o/prof.log 2>&1
