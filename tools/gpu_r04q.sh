#!/bin/bash
# Round 4: tie-break FULL kernel, weights / reliabilities staged 8 loads at a time (tbwr8, tbw8)
set -u
o=gpurun_out/r04q
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb.json 2> $o/tb.err && \
for v in tbwr8 tbw8; do
  BCE_LIB=tools/ablate_build/$v/libbce_hip.so timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 > $o/tb_$v.json 2> $o/tb_$v.err || exit 1
done && \
timeout -k 10 200 python3 bench.py --config tb --steps 20 --warmup 3 --no-cpu-baseline > $o/tb_again.json 2> $o/tb_again.err
