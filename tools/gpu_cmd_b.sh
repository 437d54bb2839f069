#!/bin/bash
# round-3 profiling call B (GPU box, repo root)
set -u
export TMPDIR=/tmp
o=gpurun_out/r03f
mkdir -p $o
timeout -k 10 400 python3 bench.py --config c3 --shard all/8 --steps 10 --warmup 2 --prewarm-s 0.2 --no-cpu-baseline > $o/c3_shards.json 2> $o/c3_shards.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/shard0 -o run --output-format csv -- python3 bench.py --config c3 --shard 0/8 --steps 10 --warmup 2 --prewarm-s 0.2 --no-cpu-baseline > $o/shard0.log 2>&1 && \
bash tools/gpu_profile.sh r03f_c3 consensus signals_this_rank=100000000 steps_total=15 stream_read_bytes=1201627112 -- --config c3 && \
bash tools/gpu_profile.sh r03f_ns namespace_resolve_kernel sources=10000000 -- --config ns && \
bash tools/gpu_profile.sh r03f_agg aggregate_kernel groups=10000 -- --config agg && \
timeout -k 10 400 python3 bench.py --config c5 --steps 6 --warmup 1 --prewarm-s 0.3 > $o/c5.json 2> $o/c5.err && \
timeout -k 10 400 python3 bench.py --config c3 --steps 30 --warmup 5 > $o/c3.json 2> $o/c3.err
