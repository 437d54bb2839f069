#!/bin/bash
# GPU box, repo root: refresh after the LDS exp table (decay kernels) -- every -m gpu test, smoke(), the
# default bench (headline + secondary lines), C3 shards, rocprof stats + PMC for C3.
set -u
o=gpurun_out/r03z4
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $o/smoke.txt 2>&1 && \
timeout -k 10 500 python3 bench.py > $o/default.json 2> $o/default.err && \
timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/c3_shards.json 2> $o/c3_shards.err && \
bash tools/gpu_profile.sh c3 consensus signals_this_rank=100000000 steps_total=15 -- --config c3
