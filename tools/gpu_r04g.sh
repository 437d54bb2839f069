#!/bin/bash
# Round 4 evidence on the final tree: every -m gpu test, smoke, the default bench (headline +
# secondary lines), ns / agg lines, C3 shard steps, the f2 front end.  rocprof stats + PMC per
# line: tools/gpu_prof_all.sh, a call of its own (the two together exceed one call's limit).
set -u
o=gpurun_out/r04g
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest_gpu.txt 2>&1 && \
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > $o/smoke.txt 2>&1 && \
timeout -k 10 400 python3 bench.py > $o/default.json 2> $o/default.err && \
timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 > $o/ns.json 2> $o/ns.err && \
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg.json 2> $o/agg.err && \
timeout -k 10 240 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/c3_shards.json 2> $o/c3_shards.err && \
timeout -k 10 300 python3 tools/bench_jsonl.py --reps 3 > $o/f2_jsonl.json 2> $o/f2_jsonl.err
