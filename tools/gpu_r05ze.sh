#!/bin/bash
# Round 5: C3 FAST full batch -- np2 bins in their own launches (shipped) vs 2049..3072 always
# in the 8-wave launch (mergehi) vs both np2 bins merged (mergeall); 1M and 10M sources.
set -u
o=gpurun_out/r05ze
mkdir -p $o
export TMPDIR=/tmp
for rep in 1 2; do
  for v in ship mergehi mergeall; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05ze] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c3 --single-mode --no-cpu-baseline --no-parity --steps 30 --warmup 5 \
      > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --c3-sources 10000000 --single-mode --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      > $o/c3S10M_${v}_$rep.json 2> $o/c3S10M_${v}_$rep.err || exit $?
  done
done
