#!/bin/bash
# Round 5 A/B: LDS-DMA prefetch of the FAST per-unique relconf / present-bit rows (kWideDma,
# shipped lib) vs register gathers (tools/bin/variants/nodma).  Parity first (shipped lib), then
# C3 FAST single-mode, C3 shards and C3 over a 10M-source table, interleaved ship / nodma.
set -u
o=gpurun_out/r05i
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_wide.py tests/test_gpu_sharded.py tests/test_gpu_consensus.py > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship nodma; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/nodma/libbce_hip.so; fi
    echo "[r05i] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline --no-parity --single-mode \
      > $o/c3_${v}_$rep.json 2> $o/c3_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --shard all/8 --steps 30 --warmup 5 --no-cpu-baseline --no-parity \
      > $o/shards_${v}_$rep.json 2> $o/shards_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --c3-sources 10000000 --steps 20 --warmup 3 --no-cpu-baseline --no-parity --single-mode \
      > $o/c3S10M_${v}_$rep.json 2> $o/c3S10M_${v}_$rep.err || exit $?
  done
done
unset BCE_LIB
