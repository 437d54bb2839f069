#!/bin/bash
# Round 5: C4 replay step and f3 namespace pass with XCD-contiguous block numbering (shipped)
# vs launch order (ewnoxcd), three interleaved reps; the drop-in / namespace GPU tests first.
set -u
o=gpurun_out/r05zs
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_namespace_aggregate.py tests/test_gpu_dropin.py -m gpu \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship ewnoxcd; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zs] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline > $o/c4_${v}_$rep.json 2> $o/c4_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns_${v}_$rep.json 2> $o/ns_${v}_$rep.err || exit $?
  done
done
