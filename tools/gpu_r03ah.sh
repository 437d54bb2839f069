#!/bin/bash
# C4 replay step: exp table staged in LDS (product build) vs the constant-table gather (whead)
set -u
o=gpurun_out/r03ah
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_dropin.txt 2>&1 && \
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline > $o/c4_lds_$k.json 2> $o/c4_lds_$k.err || exit 1
  BCE_LIB=tools/ablate_build/whead/libbce_hip.so timeout -k 10 200 python3 bench.py --config c4 --steps 200 --warmup 20 --no-cpu-baseline > $o/c4_glob_$k.json 2> $o/c4_glob_$k.err || exit 1
done
