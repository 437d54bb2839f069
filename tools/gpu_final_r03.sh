#!/bin/bash
# GPU box, repo root: round-3 evidence in one call -- every -m gpu test, smoke(), the default
# bench (headline + c3/c4/tb/c5 secondary lines), the f3/f4 lines, the C3 shard prediction,
# then rocprof stats + PMC for C2 and C3.  Stops at the first failing step.
set -u
o=gpurun_out/r03z
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $o/smoke.txt 2>&1 && \
timeout -k 10 500 python3 bench.py > $o/default.json 2> $o/default.err && \
timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 > $o/ns.json 2> $o/ns.err && \
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg.json 2> $o/agg.err && \
timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/c3_shards.json 2> $o/c3_shards.err && \
bash tools/gpu_profile.sh c2 consensus_tab32_kernel markets=1000000 signals_per_market=32 kernel=consensus_tab32_kernel -- --no-secondary && \
bash tools/gpu_profile.sh c3 consensus signals_this_rank=100000000 steps_total=15 -- --config c3
