#!/bin/bash
# Round 4: C3 launch structure -- HIP-graph replay of the planned step (1 GPU and the 8-shard
# prediction), per-bin vs team kernel, a kernel trace of one shard's steps; f2 front end.
set -u
o=gpurun_out/r04d
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity > $o/c3.json 2> $o/c3.err && \
timeout -k 10 200 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity --graph > $o/c3_graph.json 2> $o/c3_graph.err && \
timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/shards.json 2> $o/shards.err && \
timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 --graph > $o/shards_graph.json 2> $o/shards_graph.err && \
BCE_WIDE_TEAM=1 timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 --graph > $o/shards_team_graph.json 2> $o/shards_team_graph.err && \
BCE_WIDE_TEAM=1 BCE_LIB=tools/ablate_build/tless/libbce_hip.so timeout -k 10 200 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 --graph > $o/shards_tless_graph.json 2> $o/shards_tless_graph.err && \
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/trace -o run --output-format csv -- \
  python3 bench.py --config c3 --shard 0/8 --steps 10 --warmup 2 --prewarm-s 0.2 > $o/trace.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace -d $o/trace_graph -o run --output-format csv -- \
  python3 bench.py --config c3 --shard 0/8 --steps 10 --warmup 2 --prewarm-s 0.2 --graph > $o/trace_graph.log 2>&1 && \
timeout -k 10 300 python3 tools/bench_jsonl.py --reps 3 > $o/f2_jsonl.json 2> $o/f2_jsonl.err
