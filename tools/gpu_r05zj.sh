#!/bin/bash
# Round 5: C5 with 1024-thread exact / 512-thread MFMA workgroups -- reestimate GPU tests and the
# default c5 line (exact main mode + the mfma pass beside it, parity on).
set -u
o=gpurun_out/r05zj
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin.py -k "reestimate or agreement" \
  > $o/pytest.txt 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c5 --steps 8 --warmup 2 > $o/c5.json 2> $o/c5.err || exit $?
timeout -k 10 300 python3 bench.py --config c5 --mode mfma --single-mode --no-parity --no-cpu-baseline --steps 8 --warmup 2 > $o/c5_mfma.json 2> $o/c5_mfma.err
