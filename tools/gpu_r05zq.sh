#!/bin/bash
# Round 5: C2 headline -- tab kernel with XCD-contiguous block numbering (shipped) vs launch
# order (tabnoxcd), three interleaved reps; the consensus GPU tests first.
set -u
o=gpurun_out/r05zq
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_consensus.py \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship tabnoxcd; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zq] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --no-secondary --no-cpu-baseline --steps 200 --warmup 20 > $o/c2_${v}_$rep.json 2> $o/c2_${v}_$rep.err || exit $?
  done
done
