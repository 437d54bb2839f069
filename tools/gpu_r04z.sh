#!/bin/bash
# Round 4: C3 with the side stream (short-market bins) at low / high priority vs the default.
set -u
o=gpurun_out/r04z
mkdir -p $o
export TMPDIR=/tmp
python3 -c "import torch; print(torch.cuda.is_available())" > /dev/null
timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3.json 2> $o/c3.err && \
BCE_SIDE_PRIO=low timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3_low.json 2> $o/c3_low.err && \
BCE_SIDE_PRIO=high timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3_high.json 2> $o/c3_high.err && \
BCE_SIDE_PRIO=low timeout -k 10 240 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/c3_shards_low.json 2> $o/c3_shards_low.err && \
timeout -k 10 240 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 > $o/c3_shards.json 2> $o/c3_shards.err && \
timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --single-mode > $o/c3_again.json 2> $o/c3_again.err
