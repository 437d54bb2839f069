#!/bin/bash
# Round 4: tie-break on ragged markets (1..32 agents: the general lane kernel) -- baseline for
# the general-body work; plus the uniform line again.
set -u
o=gpurun_out/r04o
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --config tb --ragged --steps 20 --warmup 3 > $o/tb_ragged.json 2> $o/tb_ragged.err && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof -o tb -- python3 bench.py --config tb --ragged --steps 10 --warmup 2 --no-cpu-baseline > $o/prof.log 2>&1
