#!/bin/bash
# exp table in LDS in every decay kernel: full GPU suite, f3 (namespace) and C4 lines vs whead
set -u
o=gpurun_out/r03ai
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $o/pytest_gpu.txt 2>&1 && \
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns_lds_$k.json 2> $o/ns_lds_$k.err || exit 1
  BCE_LIB=tools/ablate_build/whead/libbce_hip.so timeout -k 10 200 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns_glob_$k.json 2> $o/ns_glob_$k.err || exit 1
done && \
timeout -k 10 200 python3 bench.py --config c4 --steps 200 --warmup 20 > $o/c4.json 2> $o/c4.err
