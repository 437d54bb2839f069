#!/bin/bash
# Round 5: C5 MFMA pass (mode="mfma") with one contiguous column slice per XCD (shipped) vs
# launch order (c5noxcd), one mode per process; the reestimate GPU tests first.
set -u
o=gpurun_out/r05zp
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin.py -k "reestimate or agreement" \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship c5noxcd; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zp] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c5 --mode mfma --single-mode --no-parity --no-cpu-baseline --steps 10 --warmup 2 \
      > $o/c5m_${v}_$rep.json 2> $o/c5m_${v}_$rep.err || exit $?
  done
done
