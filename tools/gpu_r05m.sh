#!/bin/bash
# Round 5: C5 single-read iteration, exact kernel without the SGPR spills (weights by one
# vector load + readlane, vote words by writelane, unconditional row loads) and the MFMA pass
# on the same schedule; interleaved against HEAD's stats.hip (c5head) and the MFMA pass
# on two accumulator chains (c5acc2) or without the next-batch prefetch (c5nopf).
set -u
o=gpurun_out/r05m
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin.py -k "reestimate or agreement" \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship c5head c5acc2 c5nopf; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05m] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c5 --steps 8 --warmup 2 > $o/c5_${v}_$rep.json 2> $o/c5_${v}_$rep.err || exit $?
  done
done
