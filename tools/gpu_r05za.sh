#!/bin/bash
# Round 5: f4 aggregate -- the last chunk's ordered chains after the chunk loop in asm (four
# fixed-register 4-term batches, the next read during the adds; shipped) vs the compiler's
# 8-term loop inside the chunk loop (aggnoasm) or two batches (aggb2); GPU tests first.
set -u
o=gpurun_out/r05za
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_namespace_aggregate.py -m gpu \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship aggb2 aggnoasm; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05za] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config agg --steps 100 --warmup 10 --no-cpu-baseline > $o/agg_${v}_$rep.json 2> $o/agg_${v}_$rep.err || exit $?
  done
done
