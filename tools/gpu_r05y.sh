#!/bin/bash
# Round 5: C3 -- the FAST 6-wave kernel (2049..3072) with late next-market loads at 5 waves per
# SIMD (kWideLate6, shipped) vs loads right after the keys at 4 (nolate6): FAST single-mode,
# the 8-shard step, 10M sources, EXACT; wide / sharded / consensus GPU tests first.
set -u
o=gpurun_out/r05y
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_sharded.py tests/test_gpu_consensus.py \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship nolate6; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05y] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c3 --single-mode --no-cpu-baseline --no-parity --steps 30 --warmup 5 \
      > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --shard all/8 --no-cpu-baseline --no-parity --steps 30 --warmup 5 \
      > $o/shards_${v}_$rep.json 2> $o/shards_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --c3-sources 10000000 --single-mode --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      > $o/c3S10M_${v}_$rep.json 2> $o/c3S10M_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --mode exact --single-mode --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      > $o/c3x_${v}_$rep.json 2> $o/c3x_${v}_$rep.err || exit $?
  done
done
