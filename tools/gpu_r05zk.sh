#!/bin/bash
# Round 5: C4 replay step and f3 namespace pass on 1024-thread workgroups (shipped) vs 256
# (ew256), three interleaved reps; the drop-in / namespace GPU tests first.
set -u
o=gpurun_out/r05zk
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_namespace_aggregate.py tests/test_gpu_dropin.py -m gpu \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2 3; do
  for v in ship ew256; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zk] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c4 --steps 100 --warmup 10 --no-cpu-baseline > $o/c4_${v}_$rep.json 2> $o/c4_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config ns --steps 100 --warmup 10 --no-cpu-baseline > $o/ns_${v}_$rep.json 2> $o/ns_${v}_$rep.err || exit $?
  done
done
