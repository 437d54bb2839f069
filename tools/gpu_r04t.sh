#!/bin/bash
# Round 4: namespace pass (f3) nontemporal load / store A/B.
set -u
o=gpurun_out/r04t
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns.json 2> $o/ns.err && \
for v in nsntld nsntst nsntboth; do
  BCE_LIB=tools/ablate_build/$v/libbce_hip.so timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 > $o/ns_$v.json 2> $o/ns_$v.err || exit 1
done && \
timeout -k 10 240 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns_again.json 2> $o/ns_again.err
