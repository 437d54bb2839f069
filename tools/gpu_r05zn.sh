#!/bin/bash
# Round 5: C3 -- no barrier between the sort and the leader scan, the wave-boundary run
# corrected after barrier (b) (kWideNoBarrierA, shipped) vs the barrier (barriera): FAST
# single-mode, the 8-shard step, 10M sources, EXACT; wide / sharded / consensus GPU tests
# first, full-size parity after.
set -u
o=gpurun_out/r05zn
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_sharded.py tests/test_gpu_consensus.py \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship barriera; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zn] $(date +%T) $v rep $rep" >&2
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
unset BCE_LIB
timeout -k 10 300 python3 bench.py --config c3 --steps 10 --warmup 2 > $o/c3_parity.json 2> $o/c3_parity.err
