#!/bin/bash
# Every bench line once (GPU box, repo root): headline + secondary configs, JSON under gpurun_out/.
set -u
o=gpurun_out/bench_all
mkdir -p $o
timeout -k 10 240 python3 bench.py > $o/c2.json 2> $o/c2.err && \
timeout -k 10 300 python3 bench.py --config c3 --steps 50 --warmup 10 > $o/c3.json 2> $o/c3.err && \
timeout -k 10 240 python3 bench.py --config c4 --steps 200 --warmup 20 > $o/c4.json 2> $o/c4.err && \
timeout -k 10 400 python3 bench.py --config c5 --steps 10 --warmup 3 --prewarm-s 0.5 > $o/c5.json 2> $o/c5.err && \
timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 > $o/ns.json 2> $o/ns.err && \
timeout -k 10 240 python3 bench.py --config agg --steps 100 --warmup 10 > $o/agg.json 2> $o/agg.err
