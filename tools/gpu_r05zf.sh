#!/bin/bash
# Round 5 evidence on the final tree after the f4 asm chain (call 1 of 2): every -m gpu test, smoke, the default bench
# (headline + secondary lines), ns / agg lines, C3 shard steps, the tie-break ragged line, the
# f2 front end.  rocprof stats + PMC per line: tools/gpu_prof_all.sh (call 2).
set -u
o=gpurun_out/r05zf
mkdir -p $o
bash tools/gpu_lines.sh r05zf "pytest=tests -m gpu -q" "smoke=" \
  "default=" \
  "ns=--config ns --steps 100 --warmup 10" \
  "agg=--config agg --steps 100 --warmup 10" \
  "c3_shards=--config c3 --shard all/8 --steps 30 --warmup 5" \
  "tb_ragged=--config tb --ragged --steps 20 --warmup 3" && \
timeout -k 10 300 python3 tools/bench_jsonl.py --reps 3 > $o/f2_jsonl.json 2> $o/f2_jsonl.err
