#!/bin/bash
# Round 5: C5 pass-1 kernels, one mode per process (--single-mode, no parity / CPU legs), so
# neither mode is timed behind the other: shipped stats.hip vs HEAD's (c5head, round 4's
# kernels), exact and MFMA fast, three interleaved reps.
set -u
o=gpurun_out/r05n
mkdir -p $o
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in ship c5head; do
    for m in exact fast; do
      if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
      echo "[r05n] $(date +%T) $v $m rep $rep" >&2
      timeout -k 10 300 python3 bench.py --config c5 --mode $m --single-mode --no-parity --no-cpu-baseline --steps 10 --warmup 2 \
        > $o/c5_${v}_${m}_$rep.json 2> $o/c5_${v}_${m}_$rep.err || exit $?
    done
  done
done
