#!/bin/bash
# Round 5: tie-break staged kernels with one contiguous run of tiles per XCD and grid stride
# (kTbXcd, shipped) vs blocks in launch order (tbnoxcd): 1M x 32 and the ragged line; the
# tie-break GPU tests first.
set -u
o=gpurun_out/r05zo
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu -k "tiebreak or tb" \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship tbnoxcd; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zo] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config tb --steps 30 --warmup 5 --no-cpu-baseline > $o/tb_${v}_$rep.json 2> $o/tb_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config tb --ragged --steps 20 --warmup 3 --no-cpu-baseline > $o/tbr_${v}_$rep.json 2> $o/tbr_${v}_$rep.err || exit $?
  done
done
