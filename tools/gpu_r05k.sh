#!/bin/bash
# Round 5: C5 MFMA pass (diagonal A operand, one accumulator chain, 8 waves per SIMD) vs the
# two-chain build (tools/bin/variants/c5acc2), interleaved; the reestimate GPU tests; a
# 2-rank rehearsal of the N > 1 bench path (gloo for the max-over-ranks, both ranks on cuda:0:
# per-rank parity on real hardware) for the headline and the C3 line.
set -u
o=gpurun_out/r05k
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin.py -k reestimate \
  > $o/pytest.txt 2>&1 || exit $?
for rep in 1 2; do
  for v in ship c5acc2; do
    if [ $v = ship ]; then unset BCE_LIB; else export BCE_LIB=tools/bin/variants/c5acc2/libbce_hip.so; fi
    echo "[r05k] $(date +%T) $v rep $rep" >&2
    timeout -k 10 300 python3 bench.py --config c5 --steps 4 --warmup 1 > $o/c5_${v}_$rep.json 2> $o/c5_${v}_$rep.err || exit $?
  done
done
unset BCE_LIB
timeout -k 10 400 python3 bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 --no-secondary > $o/n2_c2.json 2> $o/n2_c2.err || exit $?
timeout -k 10 400 python3 bench.py --gpus 2 --backend gloo --config c3 --steps 10 --warmup 3 > $o/n2_c3.json 2> $o/n2_c3.err || exit $?
