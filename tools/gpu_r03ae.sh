#!/bin/bash
set -u
o=gpurun_out/r03ae
mkdir -p $o
timeout -k 10 400 python3 tools/wide_variants.py run wbase wlpt wbase wlpt --modes fast,exact --reps 20 > $o/ab.txt 2>&1 && \
timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/shards_base.json 2> $o/shards_base.err && \
BCE_LIB=tools/ablate_build/wlpt/libbce_hip.so timeout -k 10 300 python3 bench.py --config c3 --shard all/8 > $o/shards_lpt.json 2> $o/shards_lpt.err
