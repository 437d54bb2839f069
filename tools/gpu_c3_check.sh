#!/bin/bash
# GPU box: lane-exchange self-test, wide/consensus parity, then the C3 bench line -> gpurun_out/
set -u
mkdir -p gpurun_out
rm -f gpurun_out/pt_wide.txt gpurun_out/c3d.json
timeout -k 10 120 python -u -m pytest tests/test_gpu_wide.py::test_lane_exchange_selftest -m gpu -x -q --timeout 60 \
  --timeout-method thread > gpurun_out/pt_self.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_consensus.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pt_wide.txt 2>&1 || exit $?
timeout -k 10 200 python bench.py --config c3 --steps 30 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/c3d.json \
  2> gpurun_out/c3d.err
