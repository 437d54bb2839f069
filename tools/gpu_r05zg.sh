#!/bin/bash
# Round 5: C3 EXACT -- the 1-wave kernels' (65..512) chains on chain_add_deep (shipped) vs the
# 8-term chain_add (nodeep1), at 1M and 10M sources, plus the shard step in exact mode; wide /
# consensus / sharded GPU tests first.
set -u
o=gpurun_out/r05zg
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_consensus.py tests/test_gpu_sharded.py \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship nodeep1; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/$v/libbce_hip.so; fi
    echo "[r05zg] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c3 --mode exact --single-mode --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      > $o/c3x_${v}_$rep.json 2> $o/c3x_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --mode exact --shard all/8 --no-cpu-baseline --no-parity --steps 20 --warmup 3 \
      > $o/shx_${v}_$rep.json 2> $o/shx_${v}_$rep.err || exit $?
    timeout -k 10 300 python3 bench.py --config c3 --c3-sources 10000000 --mode exact --single-mode --no-cpu-baseline --no-parity --steps 10 --warmup 2 \
      > $o/c3x10M_${v}_$rep.json 2> $o/c3x10M_${v}_$rep.err || exit $?
  done
done
unset BCE_LIB
timeout -k 10 300 python3 bench.py --config c3 --mode exact --single-mode --steps 10 --warmup 2 > $o/c3x_parity.json 2> $o/c3x_parity.err
